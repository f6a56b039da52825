# The SAC update: its GPU tests, grad-step timing at the runner's batch (256) and the per-rank batches of 2 / 8
# ranks, the per-kernel rocprofv3 stats of one timing run, per-block phase stamps (diagnostics build), and (with sq)
# one SQ counter pass of the SAC kernels.
# Usage: bash scripts/gpu/sac.sh TAG [notests] [sq]
. "$(dirname "$0")/common.sh"
TAG=${1:-sac}; NOTESTS=${2:-}; SQ=${3:-}
export TMPDIR=/tmp
if [ "$NOTESTS" != "notests" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_sac.py tests/test_gpu_distributed.py tests/test_gpu_rccl.py tests/test_gpu_runner_shapes.py -m gpu -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > "$O/pytest_sac_$TAG.txt" 2>&1
  rc=$?; tail -3 "$O/pytest_sac_$TAG.txt"; soft_pytest $rc pytest_sac
fi
for b in 256 128 64 32 1024; do
  timeout -k 10 200 python scripts/prof_sac.py --steps 3000 --graph 1 --batch $b > "$O/sac_time_${TAG}_b$b.txt" 2>&1
  hard $? sac_time_$b; echo "B=$b $(tail -1 "$O/sac_time_${TAG}_b$b.txt")"
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_sac_$TAG" -o run -- \
  python3 "$R/scripts/prof_sac.py" --steps 500 --graph 1 > "$O/prof_sac_$TAG.log" 2>&1; hard $? rocprof_sac
f=$(find "$O/prof_sac_$TAG" -name "*kernel_stats.csv" | head -1); cut -d, -f1-4,7 "$f" | head -12
cd "$R"
for b in 256 64; do  # per-block phase stamps of a diagnostics build (scripts/sac_phase_timing.py --build, here)
  timeout -k 10 200 python scripts/sac_phase_timing.py --variant cur --batch $b --out "$O/sac_phases_${TAG}_b$b.json" \
    > "$O/sac_phases_${TAG}_b$b.log" 2>&1; hard $? sac_phases_$b
done
cd /tmp
if [ "$SQ" = "sq" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d "$O/pmc_sac_sq_$TAG" -o run -- \
    python3 "$R/scripts/prof_sac.py" --steps 200 --graph 1 > "$O/pmc_sac_sq_$TAG.log" 2>&1; hard $? sac_sq
fi
find "$O" -name "*kernel_trace.csv" -delete
echo DONE
