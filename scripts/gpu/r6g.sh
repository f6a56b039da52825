# Round-6 call g: whole GPU suite + smoke, then the default bench line (with the C4 / C5 legs).
. "$(dirname "$0")/common.sh"
TAG=${1:-r6g}
bash scripts/gpu/suite.sh $TAG || exit $?
timeout -k 10 600 python bench.py > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err"; hard $? bench
python -c "
import json;d=json.loads(open('$O/bench_$TAG.json').read().strip().splitlines()[-1])
print('value', round(d['value']/1e6,1), 'ms', round(d['ms_per_step'],2), 'sac us', round(d['sac']['ms_per_grad_step']*1e3,2))
print('c4', {k: d['c4'][k] for k in ('grad_steps_per_s','env_ticks_per_s','decisions_per_s','sync_ms_per_loop','seconds')})
print('c5', {k: round(v['env_ticks_per_s']/1e6,1) for k, v in d['c5'].items()})
print('c2', d['c2_single_ship']['dt4']/1e9, 'policy', d['policy_stream']['env_ticks_per_s']/1e6)"
echo DONE
