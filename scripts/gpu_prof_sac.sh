# rocprofv3 kernel-trace stats of the SAC grad step. Usage: bash scripts/gpu_prof_sac.sh TAG
set -u
TAG=${1:-sac}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 300 python scripts/prof_sac.py --steps 300 > $O/sacplain_$TAG.log 2>&1 || { echo STOP plain; exit 3; }
cat $O/sacplain_$TAG.log | tail -2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sac_$TAG -o run -- python scripts/prof_sac.py --steps 300 > $O/sacprof_$TAG.log 2>&1 || { echo STOP prof; exit 3; }
f=$(find $O/prof_sac_$TAG -name '*kernel_stats.csv' | head -1); cp $f $O/sac_kernel_stats_$TAG.csv
python -c "
import csv
for r in csv.DictReader(open('$O/sac_kernel_stats_$TAG.csv')):
    print(r['Name'][:60].ljust(60), r['Calls'], r['AverageNs'], r['Percentage'])
"
echo DONE
