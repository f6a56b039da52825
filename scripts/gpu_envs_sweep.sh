# Throughput vs envs per GPU (waves per SIMD). Usage: bash scripts/gpu_envs_sweep.sh TAG
set -u
TAG=${1:-e}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for ca in sbmpc none; do for n in 4096 8192 16384 32768 65536; do
timeout -k 10 150 python bench.py --collav $ca --envs-per-gpu $n --no-cpu-baseline --sac-steps 0 --steps 30 --warmup 10 > $O/env_${TAG}_${ca}_${n}.log 2>&1 || exit 1
tail -1 $O/env_${TAG}_${ca}_${n}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ca envs $n', round(d['value']/1e6,1), 'M env-ticks/s', d['roofline']['kernel'])"
done; done
