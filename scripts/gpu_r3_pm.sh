# env GPU tests on the in-tree library, then the C3 A/B of the variants given. Usage: bash scripts/gpu_r3_pm.sh TAG X:EPW...
set -u
TAG=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_table.py tests/test_gpu_table_fullsize.py tests/test_gpu_contract.py tests/test_gpu_run_policy.py tests/test_gpu_multi_obstacle.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1
rc=$?; tail -3 $O/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_epw.sh $TAG "$@"
