# Round-1 GPU pass on HEAD: parity tests, smoke, bench lines, phase split, rocprof kernel stats.
set -u
TAG=${1:-r1f}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1; ok $? pytest
tail -4 $O/pytest_gpu_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1; hard $? smoke
tail -1 $O/smoke_$TAG.log
timeout -k 10 300 python bench.py > $O/bench_${TAG}_sbmpc.log 2>&1; hard $? bench1
tail -1 $O/bench_${TAG}_sbmpc.log
timeout -k 10 200 python bench.py --collav none --no-cpu-baseline --sac-steps 0 > $O/bench_${TAG}_none.log 2>&1; hard $? bench2
tail -1 $O/bench_${TAG}_none.log
for ca in none sbmpc; do
SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_TIMING.so timeout -k 10 120 python scripts/phase_timing.py $ca 16 > $O/phase_${TAG}_$ca.log 2>&1; hard $? phase
grep -v amdgpu.ids $O/phase_${TAG}_$ca.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $R/bench.py --steps 20 --warmup 4 --no-cpu-baseline --sac-steps 100 > $O/prof_$TAG.log 2>&1; hard $? rocprof_stats
tail -1 $O/prof_$TAG.log
find $O/prof_$TAG -name "*stats*.csv" | head
echo DONE
