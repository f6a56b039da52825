# Env-tick cost ablations (scripts/build_ablations.sh; timing only, results intentionally differ): the default
# bench (collav sbmpc) on the in-tree library and on builds without the coastline distance (NO_MAPDIST), without
# the hull-corner grounding test (NO_GROUND), and without both plus the wind (ALL3). Usage: bash scripts/gpu/abl.sh TAG
. "$(dirname "$0")/common.sh"
TAG=${1:-abl}
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M', round(d['ms_per_step'],2),'ms', round(d['env_ticks_per_decision'],1),'ticks/dec')"; }
B="--collav sbmpc --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream --no-c4 --no-c5"
timeout -k 10 200 python bench.py $B > "$O/abl_${TAG}_base.log" 2>&1; hard $? base
echo "in-tree     $(v "$O/abl_${TAG}_base.log")"
for l in NO_MAPDIST NO_GROUND NO_WIND ALL3; do
  SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$l.so timeout -k 10 200 python bench.py $B > "$O/abl_${TAG}_$l.log" 2>&1; hard $? $l
  echo "$l  $(v "$O/abl_${TAG}_$l.log")"
done
echo DONE
