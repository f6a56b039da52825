# SAC on the device: the SAC GPU tests, the bench's SAC line, and a rocprofv3 kernel-trace of the step.
# Usage: bash scripts/gpu_sac_r2.sh TAG
set -u
TAG=${1:-sac}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sac.py tests/test_gpu_distributed.py tests/test_gpu_facade.py -m gpu -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread --durations=10 > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu_$TAG.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc"; exit $rc; fi
timeout -k 10 300 python scripts/prof_sac.py --steps 500 --graph 1 > $O/sacplain_$TAG.log 2>&1 || { echo STOP plain; exit 3; }
tail -1 $O/sacplain_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sac_$TAG -o run -- python scripts/prof_sac.py --steps 300 > $O/sacprof_$TAG.log 2>&1 || { echo STOP prof; exit 3; }
f=$(find $O/prof_sac_$TAG -name '*kernel_stats.csv' | head -1)
python -c "
import csv
for r in csv.DictReader(open('$f')):
    print(r['Name'][:60].ljust(60), r['Calls'], r['AverageNs'], r['Percentage'])
"
echo DONE
