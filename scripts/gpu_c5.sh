# C5 multi-obstacle: GPU tests + bench lines K = 1 / 2 / 4. Usage: bash scripts/gpu_c5.sh TAG
set -u
TAG=${1:-c5}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi_obstacle.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $O/pytest_gpu_$TAG.log | head; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for k in 2 4; do for ca in sbmpc none; do
  timeout -k 10 300 python bench.py --obs-ships $k --collav $ca --no-cpu-baseline --sac-steps 0 --no-c2 > $O/bench_${TAG}_k${k}_$ca.log 2>&1 || { echo STOP; exit 3; }
  python -c "import json;d=json.loads(open('$O/bench_${TAG}_k${k}_$ca.log').read().strip().splitlines()[-1]);print('K=$k $ca', round(d['value']/1e6,1),'M', round(d['roofline']['kernel_ms_timed'],2),'ms')"
done; done
