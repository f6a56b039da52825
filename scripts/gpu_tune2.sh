# grid A/B, LPE sweep, SAC BLAS probe
set -u
TAG=${1:-r1b}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu_$TAG.log 2>&1; ok $? pytest
tail -4 $O/pytest_gpu_$TAG.log
B="python bench.py --no-cpu-baseline --sac-steps 0"
for ca in none sbmpc; do
  for lpe in 2 4 8 16; do
    timeout -k 10 300 $B --collav $ca --lpe $lpe > $O/t_${TAG}_${ca}_lpe$lpe.log 2>&1; hard $? bench_${ca}_${lpe}
    echo "$ca lpe$lpe grid: $(python -c "import json;d=json.loads(open('$O/t_${TAG}_${ca}_lpe$lpe.log').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M', round(d['roofline']['frac']*100,3),'%')")"
  done
  SHIPSIM_NO_GRID=1 timeout -k 10 300 $B --collav $ca > $O/t_${TAG}_${ca}_nogrid.log 2>&1; hard $? bench_nogrid
  echo "$ca lpe16 nogrid: $(python -c "import json;d=json.loads(open('$O/t_${TAG}_${ca}_nogrid.log').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M')")"
done
timeout -k 10 300 python scripts/sac_probe.py > $O/sac_probe_$TAG.log 2>&1; hard $? sac_probe
cat $O/sac_probe_$TAG.log | grep -v amdgpu.ids
echo DONE
