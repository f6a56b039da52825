#!/bin/bash
# A whole libshipsim (both objects, the product's flags) from the kernel sources of another git revision, with this
# tree's include/ (the C ABI header), for env timing A/Bs through SHIPSIM_LIB (scripts/gpu/env_abn.sh).
#   bash scripts/build_shipsim_at.sh NAME [GITREF=HEAD]  ->  ast_sac_amd/lib/abl/NAME.so
# EXTRA="flags" adds hipcc flags to every object; STRATEGY=name replaces the machine scheduler strategy.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REF=${2:-HEAD}
D=$(mktemp -d /tmp/shipsim_src.XXXX)
for f in shipsim_kernels.hip shipsim_device.hpp shipsim_diag.hpp; do
  git -C "$R" show "$REF:ast_sac_amd/csrc/$f" > "$D/$f"
done
OUT=$R/ast_sac_amd/lib/abl/$NAME.so
mkdir -p "$R/ast_sac_amd/lib/abl"
BASE="$(cd "$R" && python3 -c 'from ast_sac_amd.build_hash import HIPFLAGS; print(" ".join(f for f in HIPFLAGS if f != "-shared"))')"
OBJS=()
i=0
while IFS= read -r SET; do
  if [ -n "${STRATEGY:-}" ]; then SET=${SET//amdgpu-sched-strategy=max-ilp/amdgpu-sched-strategy=$STRATEGY}; fi
  /opt/rocm/bin/hipcc $BASE $SET ${EXTRA:-} -I"$D" -I"$R/include" -DSHIPSIM_SRC_HASH="\"variant-$NAME\"" -c "$D/shipsim_kernels.hip" \
    -o "$OUT.$i.o" &
  OBJS+=("$OUT.$i.o")
  i=$((i + 1))
done < <(cd "$R" && python3 -c 'from ast_sac_amd.build_hash import lib_flag_sets; [print(" ".join(s)) for s in lib_flag_sets("shipsim")]')
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${OBJS[@]}" -o "$OUT"
rm -f "${OBJS[@]}"
rm -rf "$D"
echo "built $OUT"
