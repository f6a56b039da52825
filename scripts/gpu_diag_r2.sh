# Diagnostics: per-phase cycle split (timing build) and the GPU parity tests on the LDS-poisoned build
# (every LDS word preset to a signalling-NaN pattern before staging). Usage: bash scripts/gpu_diag_r2.sh TAG
set -u
TAG=${1:-diag}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for ca in sbmpc none; do
  SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_TIMING.so timeout -k 10 200 python scripts/phase_timing.py $ca 16 > $O/phase_${TAG}_$ca.log 2>&1 || { echo "STOP phase $ca"; tail -3 $O/phase_${TAG}_$ca.log; exit 3; }
  grep -v amdgpu.ids $O/phase_${TAG}_$ca.log
done
SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_POISON.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_table.py tests/test_gpu_table_fullsize.py tests/test_gpu_contract.py tests/test_gpu_multi_obstacle.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_poison_$TAG.log 2>&1; rc=$?
tail -4 $O/pytest_poison_$TAG.log; echo "poison rc=$rc"
