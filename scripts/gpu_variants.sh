# SBMPC micro + sbmpc/none bench for the default lib and ablation libs given as args (lib/abl/lib_<X>.so)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in default "$@"; do
  if [ $v = default ]; then unset SHIPSIM_LIB; else export SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$v.so; fi
  timeout -k 10 120 python scripts/sbmpc_micro.py 2>&1 | grep "per pass" | sed "s/^/$v /" || { echo "FAIL micro $v"; exit 1; }
  for ca in sbmpc none; do
    timeout -k 10 150 python bench.py --collav $ca --no-cpu-baseline --sac-steps 0 > $O/var_${v}_$ca.log 2>&1 || { echo "FAIL $v $ca"; exit 1; }
    tail -1 $O/var_${v}_$ca.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $ca', round(d['value']/1e6,1), 'M')"
  done
done
