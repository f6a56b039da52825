# Collector / policy-kernel validation and the C4 loop measurement. Usage: bash scripts/gpu_r3_collector.sh TAG
set -u
TAG=${1:-r3col}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_policy_act.py tests/test_gpu_rccl.py tests/test_gpu_facade.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1
rc=$?; tail -4 $O/pytest_$TAG.log
case $rc in 0|1) ;; *) echo "STOP pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python scripts/c4_loop.py 8192 > $O/c4_loop_$TAG.json 2> $O/c4_loop_$TAG.err || { echo "c4 FAIL"; tail -5 $O/c4_loop_$TAG.err; exit 1; }
python - <<PY
import json; d=json.load(open("$O/c4_loop_$TAG.json"))
for k,v in d.items():
    if isinstance(v, dict): print(k, {a: (round(b/1e6,2) if 'per_s' in a and b>1e5 else round(b,2) if isinstance(b,float) else b) for a,b in v.items()})
PY
