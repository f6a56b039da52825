# Dynamic instruction classes per env-tick of the headline kernel: the bench line (for env-ticks per launch) and two
# rocprofv3 --pmc passes of the same command, 8 SQ counters each (scripts/pmc_classes.py).
#   bash scripts/gpu/inventory_classes.sh TAG
. "$(dirname "$0")/common.sh"
TAG=${1:-icl}
B="$R/bench.py --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream --no-c4 --no-c5 --steps 3"
timeout -k 10 300 python $B > "$O/icl_bench_$TAG.json" 2> "$O/icl_bench_$TAG.err"; hard $? bench
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT \
  SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv \
  -d "$O/icl_p1_$TAG" -o run -- python3 $B > "$O/icl_p1_$TAG.log" 2>&1; hard $? pmc1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F32 \
  SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_WAVES --output-format csv \
  -d "$O/icl_p2_$TAG" -o run -- python3 $B > "$O/icl_p2_$TAG.log" 2>&1; hard $? pmc2
cd "$R"
python scripts/pmc_classes.py "$O/icl_classes_$TAG.json" "$O/icl_bench_$TAG.json" "$O/icl_p1_$TAG" "$O/icl_p2_$TAG"
hard $? classes
find "$O" -name "*kernel_trace.csv" -delete
