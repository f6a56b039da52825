# Shared helpers of the GPU drivers (sourced). Every GPU step runs under its own time limit and the driver
# stops at the first failure, crash or time-out (no retries).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
hard() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP rc=$rc at $2"; exit "$rc"; fi; }
# pytest's rc 1 (a failing test) is reported but not a crash; anything else (abort, segfault, time-out) stops
soft_pytest() { local rc=$1; case $rc in 0|1) ;; *) echo "STOP pytest rc=$rc at $2"; exit "$rc";; esac; }
