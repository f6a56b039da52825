set -u
TAG=${1:-r1c}; mkdir -p $GRAFT_REPO_ROOT/gpurun_out
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu_${TAG:-r1c}.log 2>&1; ok $? pytest
tail -5 $O/pytest_gpu_${TAG:-r1c}.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_${TAG:-r1c}.log 2>&1; ok $? smoke
tail -2 $O/smoke_${TAG:-r1c}.log
timeout -k 10 600 python bench.py > $O/bench_${TAG:-r1c}_sbmpc.log 2>&1; ok $? bench1
tail -2 $O/bench_${TAG:-r1c}_sbmpc.log
timeout -k 10 600 python bench.py --collav none --no-cpu-baseline > $O/bench_${TAG:-r1c}_none.log 2>&1; ok $? bench2
tail -2 $O/bench_${TAG:-r1c}_none.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_${TAG:-r1c} -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_${TAG:-r1c}.log 2>&1; ok $? rocprof
find $O/prof_${TAG:-r1c} -name "*stats*" | head
