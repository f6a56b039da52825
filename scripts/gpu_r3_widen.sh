# Final-build numbers beyond the headline: C4 shard (8,192 envs/GPU) and 65,536 envs/GPU (sbmpc, none),
# C5 K = 2 / 4 (tests + bench), and the C4 loop (collector + SAC at the reference ratio).
# Usage: bash scripts/gpu_r3_widen.sh TAG
set -u
TAG=${1:-r3w}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for n in 8192 65536; do for ca in sbmpc none; do
  timeout -k 10 300 python bench.py --envs-per-gpu $n --collav $ca --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream > $O/bench_${TAG}_n${n}_$ca.log 2>&1 || { echo STOP; tail -3 $O/bench_${TAG}_n${n}_$ca.log; exit 3; }
  python -c "import json;d=json.loads(open('$O/bench_${TAG}_n${n}_$ca.log').read().strip().splitlines()[-1]);print('N=$n $ca', round(d['value']/1e6,1),'M', round(d['roofline']['kernel_ms_timed'],2),'ms lpe', d['config']['lanes_per_env'])"
done; done
bash scripts/gpu_c5.sh ${TAG}c5 || exit 3
SKIP_TESTS=1 bash scripts/gpu_r3_collector.sh ${TAG}col
