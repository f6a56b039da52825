# SAC A/B on one box: grad-step timing (scripts/prof_sac.py, graph-replayed) of the in-tree libsacfused against a
# baseline build (ast_sac_amd/lib/abl/libsacfused_base.so through SACFUSED_LIB), alternating, at B = 256 and 64;
# the SAC GPU parity tests first. Usage: bash scripts/gpu/sac_ab.sh TAG [reps] [baseline name: lib/abl/libsacfused_<name>.so]
. "$(dirname "$0")/common.sh"
TAG=${1:-sab}; REPS=${2:-2}; BASE=${3:-base}
timeout -k 10 600 python -u -m pytest tests/test_sac.py -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > "$O/pytest_sac_$TAG.txt" 2>&1
rc=$?; tail -2 "$O/pytest_sac_$TAG.txt"; soft_pytest $rc pytest_sac
u() { python -c "import ast;d=ast.literal_eval(open('$1').read().strip().splitlines()[-1]);print(round(d['ms_per_grad_step']*1e3,2),'us')"; }
for i in $(seq 1 "$REPS"); do
  for b in 256 64; do
    timeout -k 10 200 python scripts/prof_sac.py --steps 3000 --graph 1 --batch $b > "$O/sab_${TAG}_new_b${b}_$i.txt" 2>&1
    hard $? new_$b
    SACFUSED_LIB=$R/ast_sac_amd/lib/abl/libsacfused_$BASE.so timeout -k 10 200 python scripts/prof_sac.py --steps 3000 \
      --graph 1 --batch $b > "$O/sab_${TAG}_base_b${b}_$i.txt" 2>&1; hard $? base_$b
    echo "rep $i B=$b: new $(u "$O/sab_${TAG}_new_b${b}_$i.txt") | base $(u "$O/sab_${TAG}_base_b${b}_$i.txt")"
  done
done
echo DONE
