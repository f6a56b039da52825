# SAC A/B over several builds on one box: the SAC GPU parity tests on the in-tree libsacfused first, then grad-step
# timing (scripts/prof_sac.py, graph-replayed) of the in-tree build and of each named variant
# (ast_sac_amd/lib/abl/libsacfused_<name>.so through SACFUSED_LIB, built by scripts/build_sac_variant.sh), alternating,
# at B = 256 and 64.  Usage: bash scripts/gpu/sac_abn.sh TAG REPS name1 [name2 ...]   (TESTS=0 skips the tests)
. "$(dirname "$0")/common.sh"
TAG=${1:-sabn}; REPS=${2:-2}; shift 2
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_sac.py -m gpu -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > "$O/pytest_sac_$TAG.txt" 2>&1
  rc=$?; tail -2 "$O/pytest_sac_$TAG.txt"; soft_pytest $rc pytest_sac
fi
u() { python -c "import ast;d=ast.literal_eval(open('$1').read().strip().splitlines()[-1]);print(round(d['ms_per_grad_step']*1e3,2))"; }
for i in $(seq 1 "$REPS"); do
  for b in 256 64; do
    line="rep $i B=$b:"
    for v in tree "$@"; do
      f="$O/sabn_${TAG}_${v}_b${b}_$i.txt"
      if [ "$v" = tree ]; then
        timeout -k 10 200 python scripts/prof_sac.py --steps 3000 --graph 1 --batch $b > "$f" 2>&1; hard $? "$v"_$b
      else
        SACFUSED_LIB=$R/ast_sac_amd/lib/abl/libsacfused_$v.so timeout -k 10 200 python scripts/prof_sac.py --steps 3000 \
          --graph 1 --batch $b > "$f" 2>&1; hard $? "$v"_$b
      fi
      line="$line $v $(u "$f") us |"
    done
    echo "$line"
  done
done
echo DONE
