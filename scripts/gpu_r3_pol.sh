# Policy-in-the-loop stream: its tests + the open-loop stream's, the SAC barrier A/B, then the C3 A/B
# (run_table must not pay for the policy code). Usage: bash scripts/gpu_r3_pol.sh TAG
set -u
TAG=${1:-r3pol}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_run_policy.py tests/test_gpu_table.py tests/test_gpu_policy_act.py tests/test_gpu_facade.py tests/test_sac.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1
rc=$?; tail -12 $O/pytest_$TAG.log
case $rc in 0|1) ;; *) echo "STOP pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python scripts/sac_ab.py 3000 > $O/sac_ab_$TAG.json 2> $O/sac_ab_$TAG.err || { echo "sac_ab FAIL"; tail -5 $O/sac_ab_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('$O/sac_ab_$TAG.json'))
for k,v in d.items(): print(k, round(v['grad_steps_per_s']), 'steps/s', round(v['us_per_step'],1), 'us', [round(x) for x in v['runs']], v['status'])"
bash scripts/gpu_ab_libs.sh $TAG nopol new
