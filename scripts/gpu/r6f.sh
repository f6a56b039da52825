# Round-6 call f: SAC tests + store-variant A/B of the per-mask instantiated kernels; env instruction classes (PMC).
. "$(dirname "$0")/common.sh"
TAG=${1:-r6f}
timeout -k 10 600 python -u -m pytest tests/test_sac.py -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > "$O/pytest_$TAG.txt" 2>&1
rc=$?; tail -2 "$O/pytest_$TAG.txt"; soft_pytest $rc pytest
TESTS=0 bash scripts/gpu/sac_abn.sh ${TAG}s 2 curwt0 curwt7c curwt6c || exit $?
bash scripts/gpu/inventory_classes.sh $TAG || exit $?
echo DONE
