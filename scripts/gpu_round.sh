# Round GPU pass: parity tests, smoke, bench lines, rocprof kernel stats + PMC traffic passes.
set -u
TAG=${1:-r1}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu_$TAG.log 2>&1; ok $? pytest
tail -8 $O/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1; hard $? smoke
tail -2 $O/smoke_$TAG.log
timeout -k 10 600 python bench.py > $O/bench_${TAG}_sbmpc.log 2>&1; hard $? bench1
tail -1 $O/bench_${TAG}_sbmpc.log
timeout -k 10 600 python bench.py --collav none --no-cpu-baseline --sac-steps 0 > $O/bench_${TAG}_none.log 2>&1; hard $? bench2
tail -1 $O/bench_${TAG}_none.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $R/bench.py --steps 20 --warmup 4 --no-cpu-baseline --sac-steps 100 > $O/prof_$TAG.log 2>&1; hard $? rocprof_stats
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$TAG -o run -- python3 $R/bench.py --steps 10 --warmup 4 --no-cpu-baseline --sac-steps 0 > $O/pmc_fetch_$TAG.log 2>&1; hard $? pmc_fetch
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$TAG -o run -- python3 $R/bench.py --steps 10 --warmup 4 --no-cpu-baseline --sac-steps 0 > $O/pmc_write_$TAG.log 2>&1; hard $? pmc_write
find $O/prof_$TAG $O/pmc_fetch_$TAG $O/pmc_write_$TAG -name "*.csv" | head -20
echo DONE
