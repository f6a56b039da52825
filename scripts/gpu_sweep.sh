# Sweep slice length / lanes-per-env for the bench workload. Usage: bash scripts/gpu_sweep.sh TAG
set -u
TAG=${1:-s}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for ca in sbmpc none; do for sl in 32 64 128 256; do for lpe in 8 16; do
timeout -k 10 120 python bench.py --collav $ca --slice $sl --lpe $lpe --no-cpu-baseline --sac-steps 0 --steps 30 --warmup 10 > $O/sw_${TAG}_${ca}_${sl}_${lpe}.log 2>&1 || exit 1
tail -1 $O/sw_${TAG}_${ca}_${sl}_${lpe}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ca slice $sl lpe $lpe', round(d['value']/1e6,1), 'M env-ticks/s, ms/step', round(d['ms_per_step'],3), d['roofline']['kernel'])"
done; done; done
