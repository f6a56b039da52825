# timing / ablation builds (diagnostics only). Output: ast_sac_amd/lib/abl/*.so
set -e
cd "$(dirname "$0")/.."
mkdir -p ast_sac_amd/lib/abl
F="-O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -std=c++17 -Iinclude -Iast_sac_amd/csrc"
/opt/rocm/bin/hipcc $F -DSHIPSIM_PHASE_TIMING ast_sac_amd/csrc/shipsim_kernels.hip -o ast_sac_amd/lib/abl/lib_TIMING.so
