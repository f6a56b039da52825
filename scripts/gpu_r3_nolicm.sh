# A/B of the no-machine-LICM build (lib/abl/lib_nolicm.so) against the in-tree library, then the env
# GPU tests on it. Usage: bash scripts/gpu_r3_nolicm.sh TAG [VARIANT]
set -u
TAG=${1:-nolicm}; V=${2:-nolicm}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
bash scripts/gpu_ab_libs.sh $TAG new $V || exit 1
export SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$V.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_table.py tests/test_gpu_table_fullsize.py tests/test_gpu_contract.py tests/test_gpu_run_policy.py tests/test_gpu_multi_obstacle.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1
rc=$?; tail -3 $O/pytest_$TAG.log; exit $rc
