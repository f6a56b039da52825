# GPU pass: parity tests + quick bench lines (no CPU baseline / SAC).
# Usage: bash scripts/gpu_test_bench.sh TAG [pytest -k expression]
set -u
TAG=${1:-t}; K=${2:-}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "${KA[@]}" > $O/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -15 $O/pytest_gpu_$TAG.log; hard $rc pytest
for ca in sbmpc none; do
timeout -k 10 200 python bench.py --collav $ca --no-cpu-baseline --sac-steps 0 > $O/bench_${TAG}_$ca.log 2>&1; hard $? bench_$ca
tail -1 $O/bench_${TAG}_$ca.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ca', round(d['value']/1e6,1), 'M env-ticks/s', d['roofline']['kernel'])"
done
echo DONE
