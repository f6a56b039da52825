# SAC GPU tests + smoke, then A/B SAC grad-step lines: the product libsacfused vs lib/abl/libsac_<X>.so.
# Usage: bash scripts/gpu_sac_ab.sh TAG X...
set -u
TAG=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -k "sac or distributed or c4" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_sac_$TAG.log 2>&1; rc=$?
tail -4 $O/pytest_sac_$TAG.log; if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_sac_$TAG.log 2>&1 || { echo "STOP smoke"; tail -3 $O/smoke_sac_$TAG.log; exit 3; }
tail -1 $O/smoke_sac_$TAG.log
for v in default "$@" default; do
  if [ $v = default ]; then unset SACFUSED_LIB; else export SACFUSED_LIB=$R/ast_sac_amd/lib/abl/libsac_$v.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-c2 --steps 1 --warmup 1 --sac-steps 3000 > $O/sacab_${TAG}_$v.log 2>&1 || { echo "FAIL $v"; tail -3 $O/sacab_${TAG}_$v.log; exit 1; }
  tail -1 $O/sacab_${TAG}_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read())['sac']; print('$v', round(d['grad_steps_per_s']), 'grad-steps/s', round(1000*d['ms_per_grad_step'],2), 'us')"
done
