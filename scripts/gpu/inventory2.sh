# Memory-instruction inventory of the headline stream: per env-tick SMEM / LDS / VMEM instruction counts and their
# average in-flight levels (latency = LEVEL / INSTS), branches, instruction fetches; one rocprofv3 --pmc pass.
#   bash scripts/gpu/inventory2.sh TAG NAME   (ast_sac_amd/lib/abl/NAME.so, or "tree" for the in-tree library)
. "$(dirname "$0")/common.sh"
TAG=$1; N=$2
export TMPDIR=/tmp
if [ "$N" != tree ]; then export SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/$N.so; fi
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS \
  SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VMEM_RD SQ_WAVES --output-format csv -d "$O/inv2_${TAG}" -o run -- \
  python3 "$R/scripts/tick_inventory.py" run "$O/inv2_${TAG}.json" > "$O/inv2_${TAG}.log" 2>&1; hard $? inventory2
cd "$R"
python scripts/tick_inventory.py summarize "$O/inv2_${TAG}" "$O/inv2_${TAG}.json"
find "$O" -name "*kernel_trace.csv" -delete
