# Round-end measurement: parity tests, smoke, PMC traffic passes, bench lines, rocprof kernel stats
# of the default bench command. Usage: bash scripts/gpu_final.sh TAG
set -u
TAG=${1:-final}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1; ok $? pytest
tail -3 $O/pytest_gpu_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1; hard $? smoke
tail -1 $O/smoke_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --sac-steps 0 > $O/pmc_fetch_$TAG.log 2>&1; hard $? pmc_fetch
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --sac-steps 0 > $O/pmc_write_$TAG.log 2>&1; hard $? pmc_write
cd $R
python scripts/pmc_traffic.py $O/pmc_fetch_$TAG $O/pmc_write_$TAG profiles/round1_pmc_traffic.json 4096 > $O/pmc_traffic_$TAG.json; hard $? pmc_json
cp profiles/round1_pmc_traffic.json $O/round1_pmc_traffic.json
timeout -k 10 400 python bench.py > $O/bench_${TAG}_sbmpc.log 2>&1; hard $? bench1
tail -1 $O/bench_${TAG}_sbmpc.log
timeout -k 10 200 python bench.py --collav none --no-cpu-baseline --sac-steps 0 > $O/bench_${TAG}_none.log 2>&1; hard $? bench2
tail -1 $O/bench_${TAG}_none.log
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $R/bench.py > $O/prof_$TAG.log 2>&1; hard $? rocprof_stats
cd $R
python scripts/trace_summary.py $O/prof_$TAG $O/prof_$TAG.log $O/trace_vs_bench_$TAG.json; hard $? trace_summary
find $O -name "*kernel_trace.csv" -delete
du -sh $O
echo DONE
