# Memory-side counters of the three SAC step kernels (one rocprofv3 --pmc pass per counter group, each its own run):
# FETCH_SIZE, WRITE_SIZE, L2 hits / misses; summarised per kernel by scripts/sac_pmc_summary.py.
# Usage: bash scripts/gpu/sac_pmc.sh TAG [batch]
. "$(dirname "$0")/common.sh"
TAG=${1:-sacpmc}; BATCH=${2:-256}
export TMPDIR=/tmp
cd /tmp
P="$R/scripts/prof_sac.py --steps 200 --graph 1 --batch $BATCH"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$O/pmc_sac_${TAG}_$i" -o run -- python3 $P \
    > "$O/pmc_sac_${TAG}_$i.log" 2>&1; hard $? "sac_pmc $grp"
  i=$((i + 1))
done
cd "$R"
python scripts/sac_pmc_summary.py "$O/pmc_sac_${TAG}" 4 > "$O/pmc_sac_$TAG.json"; hard $? summary
cat "$O/pmc_sac_$TAG.json"
find "$O" -name "*kernel_trace.csv" -delete
