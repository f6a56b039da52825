# SAC: tests, A/B of the tree (P2 tile order, P1 batch hand-on after the barrier) against the r6f build, stamps.
. "$(dirname "$0")/common.sh"
TAG=${1:-r6j}
timeout -k 10 600 python -u -m pytest tests/test_sac.py -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > "$O/pytest_$TAG.txt" 2>&1
rc=$?; tail -2 "$O/pytest_$TAG.txt"; soft_pytest $rc pytest
TESTS=0 bash scripts/gpu/sac_abn.sh ${TAG}s 3 ${BASE:-r6f} || exit $?
timeout -k 10 200 python scripts/sac_phase_timing.py --variant cur --batch 256 --steps 300 --out "$O/sac_phases_${TAG}_b256.json" \
  > "$O/sac_phases_${TAG}_b256.log" 2>&1; hard $? phases
python -c "
import json;d=json.load(open('$O/sac_phases_${TAG}_b256.json'))
print('B=256', round(d['step_us'],2), d.get('gaps_us'), {k: v['span_us'] for k, v in d['kernels'].items()})
for k, v in d['kernels'].items():
  for kk, vv in v['kinds'].items():
    print('  ', k, kk, {a: round(x, 2) for a, x in vv.items() if abs(x) < 1e5 and a.endswith(('med', 'max')) and not a.startswith('entry')})
"
echo DONE
