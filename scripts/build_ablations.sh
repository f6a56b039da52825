# Ablation builds (timing diagnostics only; results intentionally differ). Output: ast_sac_amd/lib/abl/*.so
set -e
cd "$(dirname "$0")/.."
mkdir -p ast_sac_amd/lib/abl
F="-O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -std=c++17 -Iinclude -Iast_sac_amd/csrc"
for v in NO_MAPDIST NO_GROUND NO_WIND; do
  /opt/rocm/bin/hipcc $F -DSHIPSIM_ABL_$v ast_sac_amd/csrc/shipsim_kernels.hip -o ast_sac_amd/lib/abl/lib_$v.so &
done
/opt/rocm/bin/hipcc $F -DSHIPSIM_ABL_NO_MAPDIST -DSHIPSIM_ABL_NO_GROUND -DSHIPSIM_ABL_NO_WIND ast_sac_amd/csrc/shipsim_kernels.hip -o ast_sac_amd/lib/abl/lib_ALL3.so &
/opt/rocm/bin/hipcc $F -ffp-contract=fast ast_sac_amd/csrc/shipsim_kernels.hip -o ast_sac_amd/lib/abl/lib_FMA.so &
wait
