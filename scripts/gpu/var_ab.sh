# A/B of narrowed libshipsim variants (scripts/build_variant.sh -> ast_sac_amd/lib/abl/NAME.so) on one box: REPS
# alternating headline bench lines per variant, then (with sq) one SQ pass per variant (cycle split + instruction
# mix of ast_step_kernel: scripts/sq_summary.py). Usage: bash scripts/gpu/var_ab.sh TAG REPS [sq] NAME...
. "$(dirname "$0")/common.sh"
TAG=$1; REPS=$2; shift 2
SQ=0; if [ "${1:-}" = sq ]; then SQ=1; shift; fi
export TMPDIR=/tmp
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M',round(d['roofline']['kernel_ms_timed'],3),'ms')"; }
B="--collav sbmpc --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream --no-c4 --no-c5"
for i in $(seq 1 "$REPS"); do
  line="rep $i:"
  for n in "$@"; do
    SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/$n.so timeout -k 10 200 python bench.py $B > "$O/var_${TAG}_${n}_$i.log" 2>&1
    hard $? "$n rep $i"; line="$line | $n $(v "$O/var_${TAG}_${n}_$i.log")"
  done
  echo "$line"
done
if [ $SQ = 1 ]; then
  cd /tmp
  for n in "$@"; do
    SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/$n.so timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY \
      SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv \
      -d "$O/varsq_${TAG}_$n" -o run -- python3 "$R/bench.py" $B > "$O/varsq_${TAG}_$n.log" 2>&1; hard $? "sq $n"
  done
  cd "$R"
  for n in "$@"; do python scripts/sq_summary.py "$O/varsq_${TAG}_$n"; done
fi
echo DONE
