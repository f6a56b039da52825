# Env timing A/B over several libshipsim builds on one box: alternating bench lines (secondary lines off) of the
# in-tree library and of each named build (ast_sac_amd/lib/abl/<name>.so through SHIPSIM_LIB), with extra bench
# arguments.  Usage: bash scripts/gpu/env_abn.sh TAG REPS "BENCH ARGS" name1 [name2 ...]
. "$(dirname "$0")/common.sh"
TAG=${1:-eabn}; REPS=${2:-2}; ARGS=${3:-}; shift 3
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1))"; }
for i in $(seq 1 "$REPS"); do
  line="rep $i [$ARGS]:"
  for n in tree "$@"; do
    f="$O/eabn_${TAG}_${n}_$i.json"
    if [ "$n" = tree ]; then
      timeout -k 10 300 python bench.py --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream --no-c4 --no-c5 $ARGS > "$f" 2> "$f.err"
    else
      SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --sac-steps 0 --no-c2 \
        --no-policy-stream --no-c4 --no-c5 $ARGS > "$f" 2> "$f.err"
    fi
    hard $? "$n"
    line="$line $n $(v "$f") M |"
  done
  echo "$line"
done
