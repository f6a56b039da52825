# Round-2 bench record: the default bench line (C3 headline + CPU baseline + C2 + SAC), the collav-none
# line, the C4 shard (8,192 envs/GPU), C5 multi-obstacle K = 2 / 4. Usage: bash scripts/gpu_bench_r2.sh TAG
set -u
TAG=${1:-r2}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
run() { name=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/bench_${TAG}_$name.log 2>&1 || { echo "STOP $name"; exit 3; }
  python -c "import json;d=json.loads(open('$O/bench_${TAG}_$name.log').read().strip().splitlines()[-1]);print('$name', round(d['value']/1e6,1),'M', d['config'].get('lanes_per_env'), round(d['roofline']['kernel_ms_timed'],3), 'ms', (d.get('sac') or {}).get('grad_steps_per_s'))"; }
run default
run none --collav none --no-cpu-baseline --sac-steps 0 --no-c2
run c4 --envs-per-gpu 8192 --no-cpu-baseline --sac-steps 0 --no-c2
run c4none --envs-per-gpu 8192 --collav none --no-cpu-baseline --sac-steps 0 --no-c2
run k2 --obs-ships 2 --no-cpu-baseline --sac-steps 0 --no-c2
run k4 --obs-ships 4 --no-cpu-baseline --sac-steps 0 --no-c2
run k4none --obs-ships 4 --collav none --no-cpu-baseline --sac-steps 0 --no-c2
echo DONE
