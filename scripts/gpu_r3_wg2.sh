# Fused vs split Adam in the SAC step: rates, then rocprofv3 kernel stats of the split step.
set -u
TAG=${1:-wg2}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python scripts/sac_wg_ab.py 3000 > $O/sac_wg_ab_$TAG.json 2> $O/sac_wg_ab_$TAG.err || { tail -3 $O/sac_wg_ab_$TAG.err; exit 1; }
cat $O/sac_wg_ab_$TAG.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split_$TAG -o run -- python scripts/sac_wg_ab.py 300 True > $O/splitprof_$TAG.log 2>&1 || { echo STOP prof; exit 3; }
f=$(find $O/prof_split_$TAG -name '*kernel_stats.csv' | head -1)
python -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'sac_' in r['Name']: print(r['Name'][22:60].ljust(40), r['Calls'], r['AverageNs'])
"
find $O -name "*kernel_trace.csv" -delete
