#!/bin/bash
# A libsacfused variant built exactly as the product (the two objects of ast_sac_amd/build_hash.py OBJECTS, linked
# into one library) plus extra hipcc flags, for timing A/Bs through SACFUSED_LIB (scripts/gpu/sac_abn.sh).
#   bash scripts/build_sac_variant.sh NAME [extra hipcc flags]  ->  ast_sac_amd/lib/abl/libsacfused_NAME.so
# REF=<git revision> builds that revision's sac_kernels.hip (with this tree's include/) instead of the tree's;
# SRC=<file> builds that file (a patched copy, for a timing-only ablation).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT=$R/ast_sac_amd/lib/abl/libsacfused_$NAME.so
SRCF=$R/ast_sac_amd/csrc/sac_kernels.hip
if [ -n "${SRC:-}" ]; then
  SRCF=$SRC
elif [ -n "${REF:-}" ]; then
  D=$(mktemp -d /tmp/sac_src.XXXX)
  git -C "$R" show "$REF:ast_sac_amd/csrc/sac_kernels.hip" > "$D/sac_kernels.hip"
  SRCF=$D/sac_kernels.hip
fi
mkdir -p "$R/ast_sac_amd/lib/abl"
BASE="$(cd "$R" && python3 -c 'from ast_sac_amd.build_hash import HIPFLAGS; print(" ".join(f for f in HIPFLAGS if f != "-shared"))')"
OBJS=()
i=0
while IFS= read -r SET; do
  /opt/rocm/bin/hipcc $BASE $SET -I"$R/include" -I"$R/ast_sac_amd/csrc" -DSACF_SRC_HASH="\"variant-$NAME\"" "$@" -c \
    "$SRCF" -o "$OUT.$i.o" &
  OBJS+=("$OUT.$i.o")
  i=$((i + 1))
done < <(cd "$R" && python3 -c 'from ast_sac_amd.build_hash import lib_flag_sets; [print(" ".join(s)) for s in lib_flag_sets("sacfused")]')
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${OBJS[@]}" -o "$OUT"
rm -f "${OBJS[@]}"
echo "built $OUT"
