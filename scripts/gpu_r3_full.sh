# Full GPU suite, SAC step A/B (five launches / persistent), C3 bench (sbmpc, none), C4 loop.
# Usage: bash scripts/gpu_r3_full.sh TAG
set -u
TAG=${1:-r3full}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1
rc=$?; tail -6 $O/pytest_$TAG.log
case $rc in 0|1) ;; *) echo "STOP pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python scripts/sac_ab.py 3000 > $O/sac_ab_$TAG.json 2> $O/sac_ab_$TAG.err || { echo "sac_ab FAIL"; tail -5 $O/sac_ab_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('$O/sac_ab_$TAG.json'))
for k,v in d.items(): print(k, round(v['grad_steps_per_s']), 'steps/s', round(v['us_per_step'],1), 'us', [round(x) for x in v['runs']], v['status'])"
for CA in sbmpc none; do
  timeout -k 10 200 python bench.py --collav $CA --no-cpu-baseline > $O/bench_${TAG}_$CA.log 2>&1 || { echo "bench FAIL $CA"; tail -3 $O/bench_${TAG}_$CA.log; exit 1; }
  tail -1 $O/bench_${TAG}_$CA.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$CA', round(d['value']/1e6,1), 'M env-ticks/s', d.get('sac',{}).get('grad_steps_per_s'))"
done
SKIP_TESTS=1 bash scripts/gpu_r3_collector.sh $TAG
