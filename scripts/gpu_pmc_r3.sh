# PMC passes of the default bench command (HBM traffic, FP64 VALU), then the default bench line and the
# rocprofv3 kernel-trace stats of that same command. Usage: bash scripts/gpu_pmc_r3.sh TAG
set -u
TAG=${1:-pmc}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
B="$R/bench.py --no-cpu-baseline --sac-steps 0 --no-c2 --no-policy-stream"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$TAG -o run -- python3 $B > $O/pmc_fetch_$TAG.log 2>&1; hard $? pmc_fetch
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$TAG -o run -- python3 $B > $O/pmc_write_$TAG.log 2>&1; hard $? pmc_write
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/pmc_fp64_$TAG -o run -- python3 $B > $O/pmc_fp64_$TAG.log 2>&1; hard $? pmc_fp64
cd $R
python scripts/pmc_traffic.py $O/pmc_fetch_$TAG $O/pmc_write_$TAG profiles/round3_pmc_traffic.json 4096 > $O/pmc_traffic_$TAG.json; hard $? pmc_json
python scripts/pmc_fp64.py $O/pmc_fp64_$TAG profiles/round3_pmc_fp64.json sbmpc 4096 4096 > $O/pmc_fp64_$TAG.json; hard $? fp64_json
cp profiles/round3_pmc_traffic.json profiles/round3_pmc_fp64.json $O/
timeout -k 10 400 python bench.py > $O/bench_${TAG}.log 2>&1; hard $? bench
tail -1 $O/bench_${TAG}.log
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $R/bench.py > $O/prof_$TAG.log 2>&1; hard $? rocprof_stats
cd $R
python scripts/trace_summary.py $O/prof_$TAG $O/prof_$TAG.log $O/trace_vs_bench_$TAG.json; hard $? trace_summary
find $O -name "*kernel_trace.csv" -delete
echo DONE
