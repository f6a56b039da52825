# Fresh-box validation of the tree as built here: GPU parity suite, smoke, the default bench line and a
# rocprofv3 kernel-stats run of the same command. Usage: bash scripts/gpu_validate.sh TAG
set -u
TAG=${1:-v}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -4 $O/pytest_gpu_$TAG.log; hard $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1; hard $? smoke
tail -1 $O/smoke_$TAG.log
timeout -k 10 400 python bench.py > $O/bench_${TAG}_sbmpc.log 2>&1; hard $? bench
tail -1 $O/bench_${TAG}_sbmpc.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof_$TAG.log 2>&1; hard $? rocprof_stats
cd $R
python scripts/trace_summary.py $O/prof_$TAG $O/prof_$TAG.log $O/trace_vs_bench_$TAG.json; hard $? trace_summary
find $O -name "*kernel_trace.csv" -delete
echo DONE
