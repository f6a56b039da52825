# Round-3 validation: full GPU suite on the in-tree build, the env parity/contract tests on the ILP-scheduler
# build of the same sources (lib/abl/lib_ilp.so: the round-2 fault reproducer), then the C3 bench A/B.
# Usage: bash scripts/gpu_r3_validate.sh TAG
set -u
TAG=${1:-r3v}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1
rc=$?; tail -4 $O/pytest_$TAG.log
case $rc in 0|1) ;; *) echo "STOP pytest rc=$rc"; exit $rc;; esac
SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_ilp.so timeout -k 10 500 python -u -m pytest tests/test_gpu_contract.py tests/test_gpu_table.py tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_${TAG}_ilp.log 2>&1
rc=$?; echo "ILP build:"; tail -3 $O/pytest_${TAG}_ilp.log
case $rc in 0|1) ;; *) echo "STOP ilp rc=$rc"; exit $rc;; esac
bash scripts/gpu_ab_libs.sh $TAG base new
