set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
run() { timeout -k 10 120 python scripts/time_lib.py "$@" 2>/dev/null | tail -1; rc=$?; if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi; }
for lib in "" abl/lib_NO_MAPDIST.so abl/lib_NO_GROUND.so abl/lib_NO_WIND.so abl/lib_ALL3.so abl/lib_FMA.so; do
  if [ -n "$lib" ]; then export SHIPSIM_LIB=$R/ast_sac_amd/lib/$lib; else unset SHIPSIM_LIB; fi
  run none 8 4096 32
done
unset SHIPSIM_LIB
run sbmpc 8 4096 32
run sbmpc 16 4096 32
run sbmpc 16 4096 64
run none 16 4096 32
run none 8 16384 32
run sbmpc 16 16384 32
