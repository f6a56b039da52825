# Register usage / spills of a narrowed build (the whole-library report: python scripts/register_report.py).
#   bash scripts/regcheck.sh [N] [extra hipcc flags]   libshipsim with -DSHIPSIM_REGCHECK=N (one kernel set):
#     N = 1 (default): the headline stream kernels (chained, LPE 16, detailed; sbmpc and none)
#     N = 2: the LPE-8 stream kernels (the C4 shard's collector: policy and table streams)
#     N = 3: the multi-obstacle (K > 1) step kernels
#   bash scripts/regcheck.sh sac H [extra hipcc flags]   libsacfused's kernels of hidden width H only
set -e
cd "$(dirname "$0")/.."
N=${1:-1}; shift || true
FLAGS="-O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -std=c++17 -Iinclude -Iast_sac_amd/csrc"
if [ "$N" = sac ]; then
  H=${1:-256}; shift || true
  /opt/rocm/bin/hipcc $FLAGS -DSACF_REGCHECK_H=$H -Rpass-analysis=kernel-resource-usage "$@" \
    ast_sac_amd/csrc/sac_kernels.hip -o /tmp/regcheck_sac.so 2> /tmp/regcheck_sac.txt
  python3 scripts/regsummary.py /tmp/regcheck_sac.txt
  exit 0
fi
/opt/rocm/bin/hipcc $FLAGS -mllvm -disable-machine-licm -mllvm -amdgpu-sched-strategy=max-ilp -mllvm -amdgpu-use-amdgpu-trackers -DSHIPSIM_REGCHECK=$N -Rpass-analysis=kernel-resource-usage "$@" \
  ast_sac_amd/csrc/shipsim_kernels.hip -o /tmp/regcheck.so 2> /tmp/regcheck.txt
python3 scripts/regsummary.py /tmp/regcheck.txt | grep -E "ast_step|sbmpc_eval|legacy"
