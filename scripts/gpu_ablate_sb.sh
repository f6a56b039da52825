# SBMPC cost split (timing diagnostics; ablated builds compute different results): default build vs
# lib/abl/lib_<X>.so, collav sbmpc. Usage: bash scripts/gpu_ablate_sb.sh X...
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for v in default "$@"; do
  if [ $v = default ]; then unset SHIPSIM_LIB; else export SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_$v.so; fi
  timeout -k 10 150 python bench.py --collav sbmpc --no-cpu-baseline --sac-steps 0 --no-c2 > $O/ablsb_${v}.log 2>&1 || { echo "FAIL $v"; tail -3 $O/ablsb_${v}.log; exit 1; }
  tail -1 $O/ablsb_${v}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']/1e6,1), 'M', round(d['roofline']['kernel_ms_timed'],3), 'ms')"
done
