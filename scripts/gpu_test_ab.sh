# GPU parity suite, then A/B bench lines: the product build vs lib/abl/lib_<X>.so (diagnostic builds of
# the same sources), collav sbmpc. Usage: bash scripts/gpu_test_ab.sh TAG X...
set -u
TAG=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -6 $O/pytest_gpu_$TAG.log; if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; exit $rc; fi
for v in default "$@" default; do
  if [ $v = default ]; then unset SHIPSIM_LIB; else export SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$v.so; fi
  timeout -k 10 150 python bench.py --collav sbmpc --no-cpu-baseline --sac-steps 0 --no-c2 > $O/ab_${TAG}_${v}.log 2>&1 || { echo "FAIL $v"; tail -3 $O/ab_${TAG}_${v}.log; exit 1; }
  tail -1 $O/ab_${TAG}_${v}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']/1e6,1), 'M', round(d['roofline']['kernel_ms_timed'],3), 'ms')"
done
