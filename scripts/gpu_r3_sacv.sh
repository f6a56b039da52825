# SAC GPU tests on lib/abl/libsac_<X>.so (a candidate), then grad-step rates at B = 256 / 1024 of the product vs it.
# Usage: bash scripts/gpu_r3_sacv.sh TAG X
set -u
TAG=$1; X=$2; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
SACFUSED_LIB=$R/ast_sac_amd/lib/abl/libsac_$X.so timeout -k 10 500 python -u -m pytest tests/test_sac.py tests/test_gpu_distributed.py tests/test_gpu_rccl.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_sacv_$TAG.log 2>&1
rc=$?; tail -2 $O/pytest_sacv_$TAG.log; if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; exit $rc; fi
for v in default $X default $X; do
  if [ $v = default ]; then unset SACFUSED_LIB; else export SACFUSED_LIB=$R/ast_sac_amd/lib/abl/libsac_$v.so; fi
  for b in 256 1024; do
    echo -n "$v B=$b: "; timeout -k 10 200 python scripts/prof_sac.py --steps 500 --graph 1 --batch $b 2>&1 | tail -1 | cut -c1-120 || exit 3
  done
done
