# Launch tail on the policy stream (shipsim_run_policy): its parity test and the collector tests, then the
# bench's policy_stream line with the tail (--tail-ticks 1024, the default) and without (0), alternating, then
# the C4 loop (its fused sweep includes 1024-tick passes with a 512 / 1024 tail). Usage: bash scripts/gpu/ptail.sh TAG
. "$(dirname "$0")/common.sh"
TAG=${1:-pt}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_run_policy.py tests/test_gpu_policy_act.py > "$O/pt_pytest_$TAG.txt" 2>&1
soft_pytest $? pytest; tail -3 "$O/pt_pytest_$TAG.txt"
p() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);s=d['extra']['policy_stream'] if 'extra' in d else d['policy_stream'];print(round(s['env_ticks_per_s']/1e6,1),'M', round(s['kernel_ms'],2),'ms')"; }
B="--collav sbmpc --no-cpu-baseline --sac-steps 0 --no-c2"
for i in 1 2; do
  timeout -k 10 200 python bench.py $B > "$O/pt_${TAG}_tail_$i.log" 2>&1; hard $? tail
  timeout -k 10 200 python bench.py $B --tail-ticks 0 > "$O/pt_${TAG}_notail_$i.log" 2>&1; hard $? notail
  echo "rep $i: policy stream tail $(p "$O/pt_${TAG}_tail_$i.log") | no tail $(p "$O/pt_${TAG}_notail_$i.log")"
done
timeout -k 10 500 python scripts/c4_loop.py 8192 > "$O/c4_loop_$TAG.json" 2> "$O/c4_loop_$TAG.err"; hard $? c4_loop
python -c "import json;d=json.load(open('$O/c4_loop_$TAG.json'));[print(k, round(v['env_ticks_per_s']/1e6,1),'M') for k,v in d.items() if k.startswith('collect')]"
echo DONE
