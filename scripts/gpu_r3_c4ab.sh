# C4 loop (fused / sliced collector, SAC, runner ratio) + C3 A/B of the in-tree library vs the
# no-policy-stream build. Usage: bash scripts/gpu_r3_c4ab.sh TAG
set -u
TAG=${1:-r3c4}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
SKIP_TESTS=1 bash scripts/gpu_r3_collector.sh $TAG || exit 1
bash scripts/gpu_ab_libs.sh $TAG nopol new
