# Round-2 iteration: all GPU tests (not -x: see every failure), then the bench lines.
# Usage: bash scripts/gpu_r2.sh TAG [pytest selection]
set -u
TAG=${1:-r2}; SEL=${2:-tests}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest $SEL -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  --durations=15 > $O/pytest_gpu_$TAG.log 2>&1; ok $? pytest
grep -E "passed|failed|FAILED|Error|perturbed" $O/pytest_gpu_$TAG.log | head -40
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M', round(d['roofline']['frac']*100,3),'%', d['roofline']['kernel_ms_timed'])"; }
for ca in sbmpc none; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --sac-steps 0 --no-c2 --collav $ca > $O/t_${TAG}_${ca}.log 2>&1; hard $? bench_$ca
  echo "$ca: $(v $O/t_${TAG}_${ca}.log)"
done
echo DONE
