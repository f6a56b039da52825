# tests (incl. HIP SAC), grid A/B, LPE sweep, SAC bench
set -u
TAG=${1:-r1c}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $O/pytest_gpu_$TAG.log 2>&1; ok $? pytest
tail -4 $O/pytest_gpu_$TAG.log
B="python bench.py --no-cpu-baseline --sac-steps 0"
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M', round(d['roofline']['frac']*100,3),'%')"; }
for ca in none sbmpc; do
  for lpe in 2 4 8 16; do
    timeout -k 10 300 $B --collav $ca --lpe $lpe > $O/t_${TAG}_${ca}_lpe$lpe.log 2>&1; hard $? bench_${ca}_${lpe}
    echo "$ca lpe$lpe grid: $(v $O/t_${TAG}_${ca}_lpe$lpe.log)"
  done
  SHIPSIM_NO_GRID=1 timeout -k 10 300 $B --collav $ca > $O/t_${TAG}_${ca}_nogrid.log 2>&1; hard $? bench_nogrid
  echo "$ca lpe16 nogrid: $(v $O/t_${TAG}_${ca}_nogrid.log)"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --sac-steps 500 > $O/sac_$TAG.log 2>&1; hard $? sac
tail -1 $O/sac_$TAG.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['sac'])"
echo DONE
