# SAC kernels: the SAC GPU tests, the phase breakdown (timing build), the grad-step rate at B = 64/256/1024.
set -u; O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O; cd $GRAFT_REPO_ROOT
TAG=${1:-ph}
timeout -k 10 600 python -u -m pytest tests/test_sac.py tests/test_gpu_distributed.py -m gpu -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $O/pytest_gpu_$TAG.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc"; exit $rc; fi
timeout -k 10 200 python scripts/sac_phase_timing.py 256 > $O/phase256_$TAG.log 2>&1 && grep -v amdgpu.ids $O/phase256_$TAG.log &&
for b in 64 256 1024; do timeout -k 10 200 python scripts/prof_sac.py --steps 500 --graph 1 --batch $b 2>&1 | tail -1 | cut -c1-110 || exit 3; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sac_$TAG -o run -- python scripts/prof_sac.py --steps 300 --graph 1 > $O/sacprof_$TAG.log 2>&1 || { echo STOP prof; exit 3; }
f=$(find $O/prof_sac_$TAG -name '*kernel_stats.csv' | head -1)
python -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'sac_' in r['Name']: print(r['Name'][22:60].ljust(40), r['Calls'], r['AverageNs'])
"
