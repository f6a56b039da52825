# Round-6 call d: the K = 2 stream with SBMPC never requested (narrowed builds), SAC bit-mask A/B and phase stamps,
# the counter list of this pool's rocprofv3.
. "$(dirname "$0")/common.sh"
TAG=${1:-r6d}
cd /tmp && timeout -k 10 60 rocprofv3 --list-avail > "$O/rocprof_avail_$TAG.txt" 2>&1; cd "$R"
grep -E "SQ_INSTS_VALU|SQ_INSTS_SALU|SQ_INSTS_SMEM|SQ_INSTS_LDS|SQ_INSTS_BRANCH|SQ_INST_" "$O/rocprof_avail_$TAG.txt" | head -60
bash scripts/gpu/env_abn.sh ${TAG}k2 1 "--obs-ships 2" k3cur sbnever3 || exit $?
TESTS=0 bash scripts/gpu/sac_abn.sh ${TAG}s 2 rtwt wt0 || exit $?
timeout -k 10 200 python scripts/sac_phase_timing.py --variant mask --steps 300 --out "$O/sac_phases_${TAG}_mask.json" \
  > "$O/sac_phases_${TAG}_mask.log" 2>&1; hard $? phases
python -c "import json;d=json.load(open('$O/sac_phases_${TAG}_mask.json'));print('mask', round(d['step_us'],2), d.get('gaps_us'), {k: v['span_us'] for k, v in d['kernels'].items()})"
echo DONE
