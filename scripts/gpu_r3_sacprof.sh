# rocprofv3 kernel-trace stats of the graph-replayed SAC grad step (B = 256). Usage: bash scripts/gpu_r3_sacprof.sh TAG
set -u
TAG=${1:-r3q}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sac_$TAG -o run -- python3 scripts/prof_sac.py --steps 300 --graph 1 > $O/sacprof_$TAG.log 2>&1 || { echo STOP prof; exit 3; }
f=$(find $O/prof_sac_$TAG -name '*kernel_stats.csv' | head -1); cp $f $O/sac_kernel_stats_$TAG.csv
find $O -name "*kernel_trace.csv" -delete
python3 - $O/sac_kernel_stats_$TAG.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "sac_" in r["Name"]: print(r["Name"][22:60].ljust(40), r["Calls"], r["AverageNs"])
PY
tail -2 $O/sacprof_$TAG.log
