# chained-decision mode: parity tests + bench both modes
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_table.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_table.log 2>&1; rc=$?
tail -5 $O/pytest_table.log; [ $rc -eq 0 ] || exit $rc
for mode in table step; do for ca in sbmpc none; do
  timeout -k 10 150 python bench.py --mode $mode --collav $ca --no-cpu-baseline --sac-steps 0 > $O/tb_${mode}_$ca.log 2>&1 || { echo "FAIL $mode $ca"; tail -5 $O/tb_${mode}_$ca.log; exit 1; }
  tail -1 $O/tb_${mode}_$ca.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode $ca', round(d['value']/1e6,1), 'M', d['roofline']['kernel'], round(d['env_ticks_per_decision'],1))"
done; done
