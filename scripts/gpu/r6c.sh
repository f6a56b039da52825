# Round-6 call c: K > 1 SBMPC service tests; C5 K = 2 activity counters (diagnostics build) and the K = 2 stream with
# SBMPC never requested; SAC timing of the run-time write-through mask at B = 256 / 64.
. "$(dirname "$0")/common.sh"
TAG=${1:-r6c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_sbmpc_multi.py tests/test_gpu_multi_obstacle.py tests/test_sac.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > "$O/pytest_$TAG.txt" 2>&1
rc=$?; tail -3 "$O/pytest_$TAG.txt"; soft_pytest $rc pytest
for K in 2 4; do
  SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/sbstats.so timeout -k 10 200 python scripts/sb_stats.py $K 2 > "$O/sb_stats_${TAG}_k$K.json" \
    2> "$O/sb_stats_${TAG}_k$K.err"; hard $? sb_stats_$K
  cat "$O/sb_stats_${TAG}_k$K.json"
done
bash scripts/gpu/env_abn.sh ${TAG}k2 1 "--obs-ships 2" k3cur sbnever3 || exit $?
bash scripts/gpu/env_abn.sh ${TAG}k2n 1 "--obs-ships 2 --collav none" || exit $?
TESTS=0 bash scripts/gpu/sac_abn.sh ${TAG}s 2 rtwt wt0 || exit $?
echo DONE
