set -u
TAG=${1:-r1d}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $O/pytest_gpu_$TAG.log 2>&1; ok $? pytest
tail -4 $O/pytest_gpu_$TAG.log
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M', round(d['roofline']['frac']*100,3),'%')"; }
for ca in sbmpc none; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --sac-steps 0 --collav $ca > $O/t_${TAG}_$ca.log 2>&1; hard $? bench_$ca
  echo "$ca: $(v $O/t_${TAG}_$ca.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sac_$TAG -o run -- python3 $R/scripts/sac_prof.py > $O/prof_sac_$TAG.log 2>&1; hard $? prof_sac
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_env_$TAG -o run -- python3 $R/bench.py --steps 20 --warmup 4 --no-cpu-baseline --sac-steps 0 > $O/prof_env_$TAG.log 2>&1; hard $? prof_env
echo DONE
