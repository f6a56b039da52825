# The C4 combined loop on one GPU (scripts/c4_loop.py: the runner's device experiment on the 8,192-env shard,
# policy in the loop, device replay, FusedSACTrainer at the reference's update ratio), after the collector's
# GPU tests. Usage: bash scripts/gpu/c4.sh TAG [notests]
. "$(dirname "$0")/common.sh"
TAG=${1:-c4}; NOTESTS=${2:-}
if [ "$NOTESTS" != "notests" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_policy_act.py tests/test_gpu_facade.py tests/test_gpu_c4_shard.py \
    -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$O/pytest_c4_$TAG.txt" 2>&1
  rc=$?; tail -3 "$O/pytest_c4_$TAG.txt"; soft_pytest $rc pytest_c4
fi
timeout -k 10 400 python scripts/c4_loop.py 8192 > "$O/c4_loop_$TAG.json" 2> "$O/c4_loop_$TAG.err"; hard $? c4_loop
tail -c 600 "$O/c4_loop_$TAG.json"; echo
echo DONE
