set -u; O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 200 python scripts/sac_phase_timing.py 256 > $O/phase256_x.log 2>&1; grep -v amdgpu.ids $O/phase256_x.log
