set -u; O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_c4_shard.py tests/test_gpu_facade.py -m gpu -q -s -p no:cacheprovider --timeout 600 --timeout-method thread --durations=5 > $O/pytest_gpu_c4.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error|C4 shard|assert" $O/pytest_gpu_c4.log | head -30; exit $rc
