# A/B of two env-library builds: alternating bench lines of a baseline build (ast_sac_amd/lib/abl/lib_base.so,
# loaded through SHIPSIM_LIB) and the in-tree build, collav sbmpc and none. Usage: bash scripts/gpu/env_ab.sh TAG [reps]
. "$(dirname "$0")/common.sh"
TAG=${1:-ab}; REPS=${2:-2}
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M')"; }
for i in $(seq 1 "$REPS"); do for ca in sbmpc none; do
  SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_base.so timeout -k 10 200 python bench.py --collav $ca --no-cpu-baseline \
    --sac-steps 0 --no-c2 --no-policy-stream --no-c4 --no-c5 > "$O/ab_${TAG}_base_$ca.log" 2>&1; hard $? base_$ca
  timeout -k 10 200 python bench.py --collav $ca --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream --no-c4 --no-c5 \
    > "$O/ab_${TAG}_new_$ca.log" 2>&1; hard $? new_$ca
  echo "rep $i $ca: base $(v "$O/ab_${TAG}_base_$ca.log")  new $(v "$O/ab_${TAG}_new_$ca.log")"
done; done
echo DONE
