# SAC grad-steps/s for the default libsacfused and ablation builds given as args (lib/abl/libsac_<X>.so)
set -u
R=$GRAFT_REPO_ROOT; cd $R
for v in default "$@"; do
  if [ $v = default ]; then unset SACFUSED_LIB; else export SACFUSED_LIB=$R/ast_sac_amd/lib/abl/libsac_$v.so; fi
  for rep in 1 2; do
    timeout -k 10 120 python scripts/sac_prof.py 2>&1 | grep grad_steps | python -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip()); print('$v', round(d['grad_steps_per_s']))" || exit 1
  done
done
