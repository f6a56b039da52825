# Launch-tail length A/B on the default bench (collav sbmpc): --tail-ticks 1024 (the default) vs 2048 vs 512,
# alternating. Usage: bash scripts/gpu/tail_len.sh TAG [reps]
. "$(dirname "$0")/common.sh"
TAG=${1:-tl}; REPS=${2:-2}
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M', round(d['ms_per_step'],2),'ms')"; }
B="--collav sbmpc --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream --no-c4 --no-c5"
for i in $(seq 1 "$REPS"); do
  for tt in 1024 2048 512; do
    timeout -k 10 200 python bench.py $B --tail-ticks $tt > "$O/tl_${TAG}_${tt}_$i.log" 2>&1; hard $? tail_$tt
  done
  echo "rep $i: 1024 $(v "$O/tl_${TAG}_1024_$i.log") | 2048 $(v "$O/tl_${TAG}_2048_$i.log") | 512 $(v "$O/tl_${TAG}_512_$i.log")"
done
echo DONE
