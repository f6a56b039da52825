# A/B: GPU parity tests on the in-tree library, then alternating bench lines of a baseline build
# (ast_sac_amd/lib/abl/lib_base.so) and the in-tree build. Usage: bash scripts/gpu_ab.sh TAG [reps]
set -u
TAG=${1:-ab}; REPS=${2:-2}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -3 $O/pytest_gpu_$TAG.log; hard $rc pytest
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M')"; }
for i in $(seq 1 $REPS); do for ca in sbmpc none; do
  SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_base.so timeout -k 10 200 python bench.py --collav $ca --no-cpu-baseline --sac-steps 0 --no-c2 > $O/ab_${TAG}_base_$ca.log 2>&1; hard $? base_$ca
  timeout -k 10 200 python bench.py --collav $ca --no-cpu-baseline --sac-steps 0 --no-c2 > $O/ab_${TAG}_new_$ca.log 2>&1; hard $? new_$ca
  echo "rep $i $ca: base $(v $O/ab_${TAG}_base_$ca.log)  new $(v $O/ab_${TAG}_new_$ca.log)"
done; done
echo DONE
