# Env-count sweep of the decision stream at the default 2048-tick launches (C3 per GPU = 4096,
# C4 shard = 8192 envs per GPU). Usage: bash scripts/gpu_envs_table.sh TAG
set -u
TAG=${1:-et}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M', round(d['roofline']['kernel_ms_timed'],2),'ms/launch', d['decision_log'])"; }
for ca in sbmpc none; do for n in 4096 8192 16384 65536; do
  st=8; [ $n -ge 16384 ] && st=4; [ $n -ge 65536 ] && st=2
  timeout -k 10 300 python bench.py --collav $ca --envs-per-gpu $n --steps $st --warmup 2 --no-cpu-baseline --sac-steps 0 --no-c2 > $O/${TAG}_${ca}_$n.log 2>&1; hard $? ${ca}_$n
  echo "$ca envs $n: $(v $O/${TAG}_${ca}_$n.log)"
done; done
echo DONE
