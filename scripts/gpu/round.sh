# One box, everything in order of importance (a test failure is reported and the run goes on; a crash, abort or
# time-out stops it): the whole GPU suite, smoke(), SAC timing at B = 256 / 128 / 32 / 1024 with its rocprofv3
# kernel stats and one SQ pass, the default bench line with the rocprofv3 stats of the same command, the C4 loop,
# and (time permitting) the PMC passes of the bench line's roofline.
# Usage: bash scripts/gpu/round.sh TAG
. "$(dirname "$0")/common.sh"
TAG=${1:-round}
export TMPDIR=/tmp
echo "== suite"; date +%T
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$O/pytest_gpu_$TAG.txt" 2>&1
rc=$?; tail -4 "$O/pytest_gpu_$TAG.txt"; grep -E "^FAILED|Error" "$O/pytest_gpu_$TAG.txt" | head -20; soft_pytest $rc pytest
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$TAG.txt" 2>&1
hard $? smoke; tail -2 "$O/smoke_$TAG.txt"
echo "== sac"; date +%T
for b in 256 128 64 32 1024; do
  timeout -k 10 200 python scripts/prof_sac.py --steps 3000 --graph 1 --batch $b > "$O/sac_time_${TAG}_b$b.txt" 2>&1
  hard $? sac_time_$b; echo "B=$b $(tail -1 "$O/sac_time_${TAG}_b$b.txt")"
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_sac_$TAG" -o run -- \
  python3 "$R/scripts/prof_sac.py" --steps 500 --graph 1 > "$O/prof_sac_$TAG.log" 2>&1; hard $? rocprof_sac
f=$(find "$O/prof_sac_$TAG" -name "*kernel_stats.csv" | head -1); cut -d, -f1-4,7 "$f" | head -8
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d "$O/pmc_sac_sq_$TAG" -o run -- \
  python3 "$R/scripts/prof_sac.py" --steps 200 --graph 1 > "$O/pmc_sac_sq_$TAG.log" 2>&1; hard $? sac_sq
cd "$R"
echo "== bench"; date +%T
timeout -k 10 500 python bench.py > "$O/bench_$TAG.log" 2>&1; hard $? bench
tail -1 "$O/bench_$TAG.log" | cut -c1-400
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python3 "$R/bench.py" \
  > "$O/prof_$TAG.log" 2>&1; hard $? rocprof_stats
cd "$R"
python scripts/trace_summary.py "$O/prof_$TAG" "$O/prof_$TAG.log" "$O/trace_vs_bench_$TAG.json"; hard $? trace_summary
echo "== c4"; date +%T
timeout -k 10 500 python scripts/c4_loop.py 8192 > "$O/c4_loop_$TAG.json" 2> "$O/c4_loop_$TAG.err"; hard $? c4_loop
tail -c 700 "$O/c4_loop_$TAG.json"; echo
# the bench line's PMC inputs (HBM traffic, FP64 VALU), when the call has the time left for three short passes
if [ "$SECONDS" -lt 780 ]; then
  echo "== pmc"; date +%T
  B="$R/bench.py --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream --no-c4 --no-c5"
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
find "$O" -name "*kernel_trace.csv" -delete
echo DONE; date +%T
