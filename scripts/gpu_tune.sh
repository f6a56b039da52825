set -u
TAG=${1:-tune}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu_$TAG.log 2>&1; ok $? pytest
tail -3 $O/pytest_gpu_$TAG.log
for cfg in "--lpe 2 --slice 0" "--lpe 8 --slice 0" "--lpe 8 --slice 32" "--lpe 8 --slice 16" "--lpe 4 --slice 32" "--lpe 16 --slice 32" "--lpe 8 --slice 32 --collav none" "--lpe 8 --slice 32 --envs-per-gpu 16384"; do
  timeout -k 10 300 python bench.py $cfg --no-cpu-baseline --steps 30 --warmup 10 > $O/bench_${TAG}.tmp 2>&1; ok $? "bench $cfg"
  python -c "import json,sys; d=json.loads(open('$O/bench_${TAG}.tmp').read().strip().splitlines()[-1]); print('$cfg', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'ticks/dec %.1f'%d['env_ticks_per_decision'], d['roofline']['kernel'])"
done
