# Env-kernel A/B: GPU test suite on the in-tree build, then the C3 bench (sbmpc, none) alternating between
# the in-tree library and lib/abl/lib_<X>.so. Usage: bash scripts/gpu_ab_env.sh TAG X [tests=1]
set -u
TAG=${1:-ab}; X=${2:-base}; TESTS=${3:-1}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
if [ "$TESTS" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1
  rc=$?; tail -3 $O/pytest_$TAG.log; [ $rc -ne 0 ] && { echo "STOP pytest rc=$rc"; exit $rc; }
fi
for round in 1 2; do
  for v in new $X; do
    if [ $v = new ]; then unset SHIPSIM_LIB; else export SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$v.so; fi
    for CA in sbmpc none; do
      timeout -k 10 150 python bench.py --collav $CA --no-cpu-baseline --sac-steps 0 --no-c2 > $O/ab_${TAG}_${v}_${CA}_$round.log 2>&1 || { echo "FAIL $v $CA"; tail -3 $O/ab_${TAG}_${v}_${CA}_$round.log; exit 1; }
      tail -1 $O/ab_${TAG}_${v}_${CA}_$round.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$round $v $CA', round(d['value']/1e6,1), 'M', round(d['roofline']['kernel_ms_timed'],3), 'ms')"
    done
  done
done
