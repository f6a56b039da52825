# Round-6 call l: the 2-rank gloo rehearsal of the bench line on one GPU (the C4 leg over two ranks), the C4 ratio loop.
. "$(dirname "$0")/common.sh"
TAG=${1:-r6l}
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --no-c2 --no-policy-stream --no-c5 \
  --steps 2 --sac-steps 100 > "$O/bench_gloo2_$TAG.json" 2> "$O/bench_gloo2_$TAG.err"; hard $? gloo2
python -c "
import json;d=json.loads(open('$O/bench_gloo2_$TAG.json').read().strip().splitlines()[-1])
print('ranks', d['ranks'], 'n_gpus', d['n_gpus'], 'value', round(d['value']/1e6,1))
print('c4', {k: d['c4'][k] for k in ('ranks','grad_steps_per_s','env_ticks_per_s','decisions_per_s','sync_ms_per_loop','dp_mode','global_envs')})
print('sac', d['sac']['ms_per_grad_step']*1e3, d['sac']['shape'][:60])"
timeout -k 10 500 python scripts/c4_loop.py 8192 > "$O/c4_loop_$TAG.json" 2> "$O/c4_loop_$TAG.err"; hard $? c4_loop
python -c "
import json;d=json.loads(open('$O/c4_loop_$TAG.json').read().strip().splitlines()[-1])
print('ratio', d['ratio']); print('sac', d['sac']); print('runner', d['runner'])"
echo DONE
