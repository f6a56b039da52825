# C3 bench (sbmpc, none) over (library, envs-per-wave) variants: "new" = the in-tree library, else
# lib/abl/lib_<X>.so; EPW 0 = full waves. Timing only. Usage: bash scripts/gpu_ab_epw.sh TAG X:EPW ...
set -u
TAG=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for round in 1 2; do
  for ve in "$@"; do
    v=${ve%%:*}; e=${ve##*:}
    if [ $v = new ]; then unset SHIPSIM_LIB; else export SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$v.so; fi
    export SHIPSIM_EPW=$e
    for CA in sbmpc none; do
      f=$O/ab_${TAG}_${v}_e${e}_${CA}_$round.log
      timeout -k 10 150 python bench.py --collav $CA --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream > $f 2>&1 || { echo "FAIL $v $e $CA"; tail -3 $f; exit 1; }
      tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$round $v epw=$e $CA', round(d['value']/1e6,1), 'M', round(d['roofline']['kernel_ms_timed'],3), 'ms')"
    done
  done
done
