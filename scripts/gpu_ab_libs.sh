# C3 bench (sbmpc, none) alternating between lib/abl/lib_<X>.so variants (timing only).
# Usage: bash scripts/gpu_ab_libs.sh TAG X1 X2 ...   (X = new: the in-tree library)
set -u
TAG=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for round in 1 2; do
  for v in "$@"; do
    if [ $v = new ]; then unset SHIPSIM_LIB; else export SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$v.so; fi
    for CA in sbmpc none; do
      timeout -k 10 150 python bench.py --collav $CA --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream > $O/ab_${TAG}_${v}_${CA}_$round.log 2>&1 || { echo "FAIL $v $CA"; tail -3 $O/ab_${TAG}_${v}_${CA}_$round.log; exit 1; }
      tail -1 $O/ab_${TAG}_${v}_${CA}_$round.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$round $v $CA', round(d['value']/1e6,1), 'M', round(d['roofline']['kernel_ms_timed'],3), 'ms')"
    done
  done
done
