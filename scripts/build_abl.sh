# A/B variants of libshipsim.so from the CURRENT sources (timing / fault-reproduction only; loaded with
# SHIPSIM_LIB=..., which the binding accepts without the source-hash check). Usage: bash scripts/build_abl.sh
set -eu
R=$(cd "$(dirname "$0")/.." && pwd); D=$R/ast_sac_amd/lib/abl; mkdir -p $D
F="-O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -std=c++17 -I$R/include -I$R/ast_sac_amd/csrc"
S=$R/ast_sac_amd/csrc/shipsim_kernels.hip

/opt/rocm/bin/hipcc $F -mllvm -amdgpu-sched-strategy=iterative-ilp -DSHIPSIM_SRC_HASH='"abl-ilp"' $S -o $D/lib_ilp.so &
wait
# lane / index checks compiled in (shipsim_diag_lane_faults), default scheduler and the ILP-first one
/opt/rocm/bin/hipcc $F -DSHIPSIM_LANECHECK -DSHIPSIM_SRC_HASH='"abl-lanecheck"' $S -o $D/lib_lanecheck.so &
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-sched-strategy=iterative-ilp -DSHIPSIM_LANECHECK -DSHIPSIM_SRC_HASH='"abl-ilp-lanecheck"' $S -o $D/lib_ilp_lanecheck.so &
wait
