# SQ stall split of ast_step_kernel (instruction fetch vs issue vs other waits), collav sbmpc and none.
# Usage: bash scripts/gpu_sq_env.sh TAG [lib]
set -u
TAG=${1:-sqenv}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
[ -n "${2:-}" ] && export SHIPSIM_LIB=$2
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_avail.txt 2>&1 || true
for CA in sbmpc none; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_IFETCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d $O/sq_${TAG}_$CA -o run -- python3 $R/bench.py --collav $CA --no-cpu-baseline --sac-steps 0 --no-c2 > $O/sq_${TAG}_$CA.log 2>&1 || { echo "STOP $CA"; tail -5 $O/sq_${TAG}_$CA.log; exit 3; }
done
cd $R
python scripts/sq_summary.py $O/sq_${TAG}_sbmpc $O/sq_${TAG}_none > $O/sq_${TAG}.txt; cat $O/sq_${TAG}.txt
