# SAC phase stamps of the current build (B = 256 and 64)
. "$(dirname "$0")/common.sh"
TAG=${1:-r6h}
for b in 256 64; do
timeout -k 10 200 python scripts/sac_phase_timing.py --variant cur --batch $b --steps 300 --out "$O/sac_phases_${TAG}_b$b.json" \
  > "$O/sac_phases_${TAG}_b$b.log" 2>&1; hard $? phases
python -c "
import json;d=json.load(open('$O/sac_phases_${TAG}_b$b.json'))
print('B=$b', round(d['step_us'],2), d.get('gaps_us'), {k: v['span_us'] for k, v in d['kernels'].items()})
for k, v in d['kernels'].items():
  for kk, vv in v['kinds'].items():
    print('  ', k, kk, {a: round(x, 2) for a, x in vv.items() if abs(x) < 1e5 and a.endswith(('med', 'max')) and not a.startswith('entry')})
"
done
echo DONE
