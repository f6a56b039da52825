# Phase split of ast_step_kernel (timing build). Usage: bash scripts/gpu_phase.sh TAG
set -u
TAG=${1:-p}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for ca in none sbmpc; do
SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_TIMING.so timeout -k 10 120 python scripts/phase_timing.py $ca 16 > $O/phase_${TAG}_$ca.log 2>&1 || exit 1
grep -v amdgpu.ids $O/phase_${TAG}_$ca.log
done
