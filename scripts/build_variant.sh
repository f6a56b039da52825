#!/bin/bash
# A narrowed libshipsim (the headline stream kernels only, -DSHIPSIM_REGCHECK=1: run_table / run_policy at LPE 16,
# detailed machinery) with the product's flags plus extra ones, for timing A/Bs through SHIPSIM_LIB (bench.py
# --no-c2 --no-policy-stream --sac-steps 0 runs on it).
#   bash scripts/build_variant.sh NAME [extra hipcc flags]  ->  ast_sac_amd/lib/abl/NAME.so
# SRC=<dir with shipsim_kernels.hip> builds another copy of the sources (default: the tree's).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
SRC=${SRC:-$R/ast_sac_amd/csrc}
mkdir -p "$R/ast_sac_amd/lib/abl"
F="$(cd "$R" && python3 -c 'from ast_sac_amd.build_hash import HIPFLAGS, LIB_FLAGS; print(" ".join(HIPFLAGS + LIB_FLAGS["shipsim"] + ["-mllvm", "-disable-machine-licm"]))')"
/opt/rocm/bin/hipcc $F -I"$R/include" -I"$SRC" -I"$R/ast_sac_amd/csrc" -DSHIPSIM_REGCHECK=1 -DSHIPSIM_SRC_HASH="\"variant-$NAME\"" "$@" \
  "$SRC/shipsim_kernels.hip" -o "$R/ast_sac_amd/lib/abl/$NAME.so"
