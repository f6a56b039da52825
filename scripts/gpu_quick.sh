# quick loop: GPU tests, phase timing, bench lines
set -u
TAG=${1:-q}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $O/pytest_gpu_$TAG.log 2>&1; ok $? pytest
tail -4 $O/pytest_gpu_$TAG.log
for ca in none sbmpc; do
SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_TIMING.so timeout -k 10 200 python scripts/phase_timing.py $ca 16 > $O/phase_${TAG}_${ca}.log 2>&1; hard $? phase
grep -v amdgpu.ids $O/phase_${TAG}_${ca}.log
done
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M', round(d['roofline']['frac']*100,3),'%')"; }
for ca in sbmpc none; do for lpe in 16 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --sac-steps 0 --collav $ca --lpe $lpe > $O/t_${TAG}_${ca}_$lpe.log 2>&1; hard $? bench_$ca
  echo "$ca lpe$lpe: $(v $O/t_${TAG}_${ca}_$lpe.log)"
done; done
echo DONE
