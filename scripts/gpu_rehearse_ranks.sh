# Rehearsal of the multi-rank bench path on a one-GPU box: bench.py --gpus 2 spawns two ranks (gloo,
# both on the one device: n_gpus reports 1 physical device, ranks 2). Usage: bash scripts/gpu_rehearse_ranks.sh TAG
set -u
TAG=${1:-ranks}; O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 2 --no-cpu-baseline --no-c2 --sac-steps 100 > $O/bench_ranks_$TAG.log 2>&1 || { echo STOP; tail -20 $O/bench_ranks_$TAG.log; exit 3; }
python -c "import json;d=json.loads(open('$O/bench_ranks_$TAG.log').read().strip().splitlines()[-1]);print({k:d[k] for k in ['value','n_gpus','ranks','ms_per_step']}, d['config']['global_envs'], d['sac']['global_batch'], d['sac']['batch_per_gpu'], round(d['sac']['grad_steps_per_s']))"
