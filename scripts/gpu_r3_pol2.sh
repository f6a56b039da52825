# Policy stream tests + bench line on the default build, then the lane-check battery. Usage: bash scripts/gpu_r3_pol2.sh TAG
set -u
TAG=${1:-r3pol2}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_run_policy.py tests/test_gpu_policy_act.py tests/test_gpu_facade.py tests/test_gpu_table.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1
rc=$?; tail -3 $O/pytest_$TAG.log
case $rc in 0|1) ;; *) echo "STOP pytest rc=$rc"; exit $rc;; esac
for CA in sbmpc none; do timeout -k 10 200 python bench.py --collav $CA --no-cpu-baseline --sac-steps 0 --no-c2 > $O/bench_$TAG.log 2>&1 || { echo "bench FAIL"; tail -3 $O/bench_$TAG.log; exit 1; }
tail -1 $O/bench_$TAG.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$CA table', round(d['value']/1e6,1), 'M; policy stream', round(d['policy_stream']['env_ticks_per_s']/1e6,1), 'M', round(d['policy_stream']['kernel_ms'],2), 'ms')"
cp $O/bench_$TAG.log $O/bench_${TAG}_$CA.log; done
bash scripts/gpu_r3_lanecheck.sh $TAG
