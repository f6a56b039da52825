# Late-round-3 check of a changed SAC library: full GPU suite, smoke, SAC A/B (five launches / persistent at
# B = 256 / 64 / 1024), the C4 loop. Usage: bash scripts/gpu_r3_end.sh TAG
set -u
TAG=${1:-r3end}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -3 $O/pytest_gpu_$TAG.log
case $rc in 0|1) ;; *) echo "STOP pytest rc=$rc"; exit $rc;; esac
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo "STOP smoke"; tail -3 $O/smoke_$TAG.log; exit 3; }
tail -2 $O/smoke_$TAG.log
timeout -k 10 300 python scripts/sac_ab.py 3000 > $O/sac_ab_$TAG.json 2> $O/sac_ab_$TAG.err || { echo "sac_ab FAIL"; tail -5 $O/sac_ab_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('$O/sac_ab_$TAG.json'))
for k,v in d.items(): print(k, round(v['grad_steps_per_s']), 'steps/s', round(v['us_per_step'],1), 'us', v['status'])"
SKIP_TESTS=1 bash scripts/gpu_r3_collector.sh $TAG
