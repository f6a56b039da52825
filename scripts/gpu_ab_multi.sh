# Multi-obstacle GPU tests, then A/B bench lines at K = 2 and 4 obstacle ships (sbmpc): the product
# build vs lib/abl/lib_<X>.so. Usage: bash scripts/gpu_ab_multi.sh TAG X...
set -u
TAG=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -k "multi or obstacle or sbmpc or parity" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_multi_$TAG.log 2>&1; rc=$?
tail -4 $O/pytest_multi_$TAG.log; if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; exit $rc; fi
for k in 2 4; do
for v in default "$@"; do
  if [ $v = default ]; then unset SHIPSIM_LIB; else export SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$v.so; fi
  timeout -k 10 200 python bench.py --obs-ships $k --no-cpu-baseline --sac-steps 0 --no-c2 > $O/abm_${TAG}_${k}_$v.log 2>&1 || { echo "FAIL $v"; tail -3 $O/abm_${TAG}_${k}_$v.log; exit 1; }
  tail -1 $O/abm_${TAG}_${k}_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('K=$k $v', round(d['value']/1e6,1), 'M', round(d['roofline']['kernel_ms_timed'],2), 'ms')"
done
done
