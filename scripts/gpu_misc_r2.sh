set -u; O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_sac.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu_sacH.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" $O/pytest_gpu_sacH.log | head; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 2 --no-cpu-baseline --no-c2 --sac-steps 100 > $O/bench_gloo2.log 2>&1 || { echo STOP gloo; tail -20 $O/bench_gloo2.log; exit 3; }
python -c "import json;d=json.loads(open('$O/bench_gloo2.log').read().strip().splitlines()[-1]);print({k:d[k] for k in ['value','n_gpus','ranks','config']}); print(d['sac']['global_batch'], d['sac']['batch_per_gpu'], d['sac']['grad_steps_per_s'])"
