# The env path's GPU tests on the two lane-check diagnostics builds (default and ILP-first scheduler), each
# ending with the violation read-out. Usage: bash scripts/gpu_r3_lanecheck.sh TAG
set -u
TAG=${1:-r3lc}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
T="tests/test_gpu_contract.py tests/test_gpu_table.py tests/test_gpu_parity.py tests/test_gpu_run_policy.py tests/test_gpu_zz_lanecheck_report.py"
for v in lanecheck ilp_lanecheck; do
  SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$v.so timeout -k 10 600 python -u -m pytest $T -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_${TAG}_$v.log 2>&1
  rc=$?; echo "$v:"; tail -3 $O/pytest_${TAG}_$v.log
  case $rc in 0|1) ;; *) echo "STOP rc=$rc"; exit $rc;; esac
done
