# SAC on the device: the SAC GPU tests, then the bench's SAC line alone (env lines skipped via tiny env run).
# Usage: bash scripts/gpu_sac_r2.sh TAG
set -u
TAG=${1:-sac}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_sac.py tests/test_gpu_distributed.py -m gpu -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread --durations=10 > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu_$TAG.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c2 --steps 2 --sac-steps 500 > $O/bench_$TAG.log 2>&1 || { echo "STOP bench"; exit 3; }
python -c "import json;d=json.loads(open('$O/bench_$TAG.log').read().strip().splitlines()[-1]);print(json.dumps(d.get('sac'),indent=1))"
echo DONE
