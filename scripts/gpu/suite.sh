# The round-end checks: the whole GPU test suite in one process, then smoke().
# Usage (on the GPU box): bash scripts/gpu/suite.sh TAG [pytest selection ...]
. "$(dirname "$0")/common.sh"
TAG=${1:-suite}; shift || true
SEL=${*:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$O/pytest_gpu_$TAG.txt" 2>&1
rc=$?; tail -3 "$O/pytest_gpu_$TAG.txt"; soft_pytest $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$TAG.txt" 2>&1; hard $? smoke
tail -2 "$O/smoke_$TAG.txt"
