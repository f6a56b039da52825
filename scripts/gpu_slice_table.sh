# Slice-length sweep of the decision stream (--mode table). Usage: bash scripts/gpu_slice_table.sh TAG "slice steps warmup" ...
set -u
TAG=${1:-st}; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M', round(d['roofline']['kernel_ms_timed'],3),'ms/launch', d['decision_log'])"; }
for ca in sbmpc none; do for cfg in "$@"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --collav $ca --slice $1 --steps $2 --warmup $3 --no-cpu-baseline --sac-steps 0 --no-c2 > $O/${TAG}_${ca}_$1.log 2>&1; hard $? ${ca}_$1
  echo "$ca slice $1 steps $2 warmup $3: $(v $O/${TAG}_${ca}_$1.log)"
done; done
echo DONE
