# Round-4 env A/B, collav sbmpc, alternating bench lines: the in-tree build with the launch tail (the default
# --tail-ticks 1024) and without (--tail-ticks 0), and a baseline build of the same sources before the DPP argmin
# (ast_sac_amd/lib/abl/lib_base.so through SHIPSIM_LIB, default tail). Usage: bash scripts/gpu/tail_ab.sh TAG [reps]
. "$(dirname "$0")/common.sh"
TAG=${1:-tail}; REPS=${2:-2}
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M', round(d['ms_per_step'],2),'ms')"; }
B="--collav sbmpc --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream --no-c4 --no-c5"
for i in $(seq 1 "$REPS"); do
  timeout -k 10 200 python bench.py $B > "$O/tab_${TAG}_tail_$i.log" 2>&1; hard $? tail
  timeout -k 10 200 python bench.py $B --tail-ticks 0 > "$O/tab_${TAG}_notail_$i.log" 2>&1; hard $? notail
  SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_base.so timeout -k 10 200 python bench.py $B > "$O/tab_${TAG}_base_$i.log" 2>&1
  hard $? base
  echo "rep $i: tail $(v "$O/tab_${TAG}_tail_$i.log") | no tail $(v "$O/tab_${TAG}_notail_$i.log") | LDS-permute argmin $(v "$O/tab_${TAG}_base_$i.log")"
done
echo DONE
