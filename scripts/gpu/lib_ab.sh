# A/B of env-library builds on one box: alternating default bench lines (collav sbmpc) of the in-tree build and of
# each ast_sac_amd/lib/abl/lib_<name>.so given (through SHIPSIM_LIB). Usage: bash scripts/gpu/lib_ab.sh TAG REPS name...
. "$(dirname "$0")/common.sh"
TAG=$1; REPS=$2; shift 2
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M')"; }
B="--collav sbmpc --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream --no-c4 --no-c5"
for i in $(seq 1 "$REPS"); do
  timeout -k 10 200 python bench.py $B > "$O/lab_${TAG}_tree_$i.log" 2>&1; hard $? tree
  line="rep $i: in-tree $(v "$O/lab_${TAG}_tree_$i.log")"
  for n in "$@"; do
    SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$n.so timeout -k 10 200 python bench.py $B > "$O/lab_${TAG}_${n}_$i.log" 2>&1
    hard $? $n; line="$line | $n $(v "$O/lab_${TAG}_${n}_$i.log")"
  done
  echo "$line"
done
echo DONE
