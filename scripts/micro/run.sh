# Microbenchmarks (diagnostics): build with hipcc here, then run one under rocprofv3 on the GPU box.
# Build (CPU container):  bash scripts/micro/run.sh build
# Run (GPU box):          bash scripts/micro/run.sh run colread2|colread|icache|launch|firstload
set -u
D=$(cd "$(dirname "$0")" && pwd)
if [ "${1:-}" = "build" ]; then
  for f in colread colread2 icache launch firstload; do /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 "$D/$f.hip" -o "$D/$f" || exit 1; done
  exit 0
fi
B=${2:-colread2}; O=${GRAFT_REPO_ROOT:-$D/../..}/gpurun_out/micro_$B; export TMPDIR=/tmp
timeout -k 5 60 "$D/$B" && cd /tmp && timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o run \
  -- "$D/$B" > /dev/null 2>&1 || exit 1
f=$(find "$O" -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f"; find "$O" -name "*kernel_trace.csv" -delete
