# SAC: GPU tests of the SAC path, grad-step A/B (sac_ab), phase timing of the timing build, rocprof kernel stats.
# Usage: bash scripts/gpu_r3_sac2.sh TAG
set -u
TAG=${1:-sac}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_sac.py tests/test_gpu_policy_act.py tests/test_gpu_distributed.py tests/test_gpu_rccl.py tests/test_gpu_c4_shard.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1
rc=$?; tail -3 $O/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/sac_ab.py 3000 > $O/sac_ab_$TAG.json 2> $O/sac_ab_$TAG.err || { echo "sac_ab FAIL"; tail -5 $O/sac_ab_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('$O/sac_ab_$TAG.json'))
for k,v in d.items(): print(k, round(v['grad_steps_per_s']), 'steps/s', round(v['us_per_step'],1), 'us', v['status'])"
timeout -k 10 200 python scripts/sac_phase_timing.py 256 > $O/phase256_$TAG.log 2>&1 && grep -v amdgpu.ids $O/phase256_$TAG.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sac_$TAG -o run -- python scripts/prof_sac.py --steps 300 --graph 1 > $O/sacprof_$TAG.log 2>&1 || { echo STOP prof; exit 3; }
f=$(find $O/prof_sac_$TAG -name '*kernel_stats.csv' | head -1)
python -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'sac_' in r['Name']: print(r['Name'][22:60].ljust(40), r['Calls'], r['AverageNs'])
"
find $O -name "*kernel_trace.csv" -delete
