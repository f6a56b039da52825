# Round-6 call b: K > 1 SBMPC service and multi-obstacle env tests, SAC tests, C5 A/B (K = 2 / 4, sbmpc) against the
# round-5 env build, SAC write-through variants.
. "$(dirname "$0")/common.sh"
TAG=${1:-r6b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_sbmpc_multi.py tests/test_gpu_multi_obstacle.py tests/test_sac.py \
  -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$O/pytest_$TAG.txt" 2>&1
rc=$?; tail -3 "$O/pytest_$TAG.txt"; soft_pytest $rc pytest
bash scripts/gpu/env_abn.sh ${TAG}k2 2 "--obs-ships 2" shipsim_r5 || exit $?
bash scripts/gpu/env_abn.sh ${TAG}k4 1 "--obs-ships 4" shipsim_r5 || exit $?
TESTS=0 bash scripts/gpu/sac_abn.sh ${TAG}s 2 wt3 wt6 wt2 wt0 || exit $?
for v in wt7 wt0; do
  timeout -k 10 200 python scripts/sac_phase_timing.py --variant $v --steps 300 --out "$O/sac_phases_${TAG}_$v.json" \
    > "$O/sac_phases_${TAG}_$v.log" 2>&1; hard $? phases_$v
  python -c "import json;d=json.load(open('$O/sac_phases_${TAG}_$v.json'));print('$v', round(d['step_us'],2), d.get('gaps_us'), {k: v['span_us'] for k, v in d['kernels'].items()})"
done
echo DONE
