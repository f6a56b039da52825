# Ablation builds (timing diagnostics only; results intentionally differ). Output: ast_sac_amd/lib/abl/*.so
set -e
cd "$(dirname "$0")/.."
mkdir -p ast_sac_amd/lib/abl
# the product's code-generation flags (ast_sac_amd/build_hash.py), so the builds differ only by the ablation
F="$(python -c 'from ast_sac_amd.build_hash import HIPFLAGS, LIB_FLAGS; print(" ".join(HIPFLAGS + LIB_FLAGS["shipsim"] + ["-mllvm", "-disable-machine-licm"]))') -Iinclude -Iast_sac_amd/csrc"
for v in NO_MAPDIST NO_GROUND NO_WIND; do
  /opt/rocm/bin/hipcc $F -DSHIPSIM_ABL_$v ast_sac_amd/csrc/shipsim_kernels.hip -o ast_sac_amd/lib/abl/lib_$v.so &
done
/opt/rocm/bin/hipcc $F -DSHIPSIM_ABL_NO_MAPDIST -DSHIPSIM_ABL_NO_GROUND -DSHIPSIM_ABL_NO_WIND ast_sac_amd/csrc/shipsim_kernels.hip -o ast_sac_amd/lib/abl/lib_ALL3.so &
wait
