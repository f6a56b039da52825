# Round-6 call e: SAC store / mask variants of the current source on one box; SBMPC optimiser per-request costs.
. "$(dirname "$0")/common.sh"
TAG=${1:-r6e}
timeout -k 10 300 python scripts/sbmpc_bench.py 65536 > "$O/sbmpc_bench_$TAG.json" 2> "$O/sbmpc_bench_$TAG.err"; hard $? sbmpc_bench
cat "$O/sbmpc_bench_$TAG.json"; echo
TESTS=0 bash scripts/gpu/sac_abn.sh ${TAG}s 3 curwt0 curwt7c curwt6c wt0 || exit $?
echo DONE
