# The headline measurement: the default bench line, the rocprofv3 kernel-trace stats of the same command
# (trace_summary.py checks rocprof's mean launch time against the bench's HIP events), and the PMC passes
# the bench line's roofline reads (HBM traffic: FETCH_SIZE / WRITE_SIZE; FP64 VALU: SQ counters), each pass
# a run of its own. Usage: bash scripts/gpu/bench_profile.sh TAG [pmc]
. "$(dirname "$0")/common.sh"
TAG=${1:-bench}; PMC=${2:-}
export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream --no-c4 --no-c5"
if [ -n "$PMC" ]; then
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch_$TAG" -o run -- python3 $B \
    > "$O/pmc_fetch_$TAG.log" 2>&1; hard $? pmc_fetch
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write_$TAG" -o run -- python3 $B \
    > "$O/pmc_write_$TAG.log" 2>&1; hard $? pmc_write
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F64 \
    SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES --output-format csv \
    -d "$O/pmc_fp64_$TAG" -o run -- python3 $B > "$O/pmc_fp64_$TAG.log" 2>&1; hard $? pmc_fp64
  cd "$R"
  python scripts/pmc_traffic.py "$O/pmc_fetch_$TAG" "$O/pmc_write_$TAG" "$O/pmc_traffic_$TAG.json" 4096 \
    > "$O/pmc_traffic_$TAG.out"; hard $? pmc_json
  python scripts/pmc_fp64.py "$O/pmc_fp64_$TAG" "$O/pmc_fp64_$TAG.json" sbmpc 4096 4096 > "$O/pmc_fp64_$TAG.out"
  hard $? fp64_json
fi
timeout -k 10 500 python bench.py > "$O/bench_$TAG.log" 2>&1; hard $? bench
tail -1 "$O/bench_$TAG.log"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python3 "$R/bench.py" \
  > "$O/prof_$TAG.log" 2>&1; hard $? rocprof_stats
cd "$R"
python scripts/trace_summary.py "$O/prof_$TAG" "$O/prof_$TAG.log" "$O/trace_vs_bench_$TAG.json"; hard $? trace_summary
find "$O" -name "*kernel_trace.csv" -delete
echo DONE
