# Per-env-tick SQ counters of the headline stream for narrowed libshipsim variants (one rocprofv3 --pmc pass each):
#   bash scripts/gpu/inventory.sh TAG NAME...   (ast_sac_amd/lib/abl/NAME.so from scripts/build_variant.sh)
. "$(dirname "$0")/common.sh"
TAG=$1; shift
export TMPDIR=/tmp
cd /tmp
args=""
for n in "$@"; do
  SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/$n.so timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY \
    SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv \
    -d "$O/inv_${TAG}_$n" -o run -- python3 "$R/scripts/tick_inventory.py" run "$O/inv_${TAG}_$n.json" \
    > "$O/inv_${TAG}_$n.log" 2>&1; hard $? "inventory $n"
  args="$args $O/inv_${TAG}_$n $O/inv_${TAG}_$n.json"
done
cd "$R"
python scripts/tick_inventory.py summarize $args > "$O/inventory_$TAG.json"; hard $? summarize
cat "$O/inventory_$TAG.json"
find "$O" -name "*kernel_trace.csv" -delete
