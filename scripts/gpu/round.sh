# One box, everything in order of importance (a test failure is reported and the run goes on; a crash, abort or
# time-out stops it): the whole GPU suite, smoke(), SAC timing at B = 256 / 128 / 32 / 1024 with its rocprofv3
# kernel stats, the default bench line with the rocprofv3 stats of the same command, the C4 loop.
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
find "$O" -name "*kernel_trace.csv" -delete
echo DONE; date +%T
