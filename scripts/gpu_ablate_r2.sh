# Ablation bench lines (diagnostics: the ablated builds compute different results): default build vs
# lib/abl/lib_<X>.so for each X given, sbmpc and none. Usage: bash scripts/gpu_ablate_r2.sh X...
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in default "$@"; do
  if [ $v = default ]; then unset SHIPSIM_LIB; else export SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$v.so; fi
  for ca in sbmpc none; do
    timeout -k 10 150 python bench.py --collav $ca --no-cpu-baseline --sac-steps 0 --no-c2 > $O/abl_${v}_$ca.log 2>&1 || { echo "FAIL $v $ca"; tail -3 $O/abl_${v}_$ca.log; exit 1; }
    tail -1 $O/abl_${v}_$ca.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $ca', round(d['value']/1e6,1), 'M')"
  done
done
