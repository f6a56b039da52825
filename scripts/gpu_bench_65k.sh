# 65,536 envs on one GPU (LPE 4): sbmpc and none bench lines. Usage: bash scripts/gpu_bench_65k.sh TAG
set -u
TAG=${1:-65k}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for ca in sbmpc none; do
  timeout -k 10 300 python bench.py --envs-per-gpu 65536 --collav $ca --no-cpu-baseline --sac-steps 0 --no-c2 > $O/bench_${TAG}_$ca.log 2>&1 || { echo "STOP $ca"; tail -3 $O/bench_${TAG}_$ca.log; exit 3; }
  tail -1 $O/bench_${TAG}_$ca.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ca', round(d['value']/1e6,1), 'M', d['config']['lanes_per_env'], round(d['roofline']['kernel_ms_timed'],2), 'ms')"
done
