# Round-2 sweep: decision-stream throughput vs envs per GPU and lanes per env; FP64 VALU counters.
# Usage: bash scripts/gpu_sweep_r2.sh TAG
set -u
TAG=${1:-sw}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_contract.py tests/test_gpu_distributed.py \
  -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1; ok $? pytest
tail -3 $O/pytest_gpu_$TAG.log
v() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value']/1e6,1),'M', round(d['roofline']['kernel_ms_timed'],2),'ms')"; }
for ca in sbmpc none; do for n in 4096 8192 65536; do for lpe in 16 8 4; do
  st=4; [ $n -eq 65536 ] && st=2
  timeout -k 10 300 python bench.py --no-cpu-baseline --sac-steps 0 --no-c2 --collav $ca --envs-per-gpu $n --lpe $lpe \
    --steps $st > $O/sw_${TAG}_${ca}_${n}_${lpe}.log 2>&1; hard $? bench
  echo "$ca N=$n lpe=$lpe: $(v $O/sw_${TAG}_${ca}_${n}_${lpe}.log)"
done; done; done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_$TAG.txt 2>&1; ok $? list
grep -o "SQ_INSTS_VALU[A-Z0-9_]*\|SQ_INSTS_SALU\|SQ_WAVES\|SQ_BUSY_CYCLES\|SQ_WAVE_CYCLES\|SQ_ACTIVE_INST_VALU\|SQ_INSTS_FLAT\|SQ_INSTS_LDS" $O/counters_$TAG.txt | sort -u > $O/sqlist_$TAG.txt
cat $O/sqlist_$TAG.txt | tr '\n' ' '; echo
echo DONE
