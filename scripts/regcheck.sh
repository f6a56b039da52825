# Register usage / spills of a narrowed build of libshipsim (-DSHIPSIM_REGCHECK=N instantiates only one kernel set):
#   N = 1 (default): the headline stream kernels (chained, LPE 16, detailed; sbmpc and none)
#   N = 2: the LPE-8 stream kernels (the C4 shard's collector: policy and table streams)
#   N = 3: the multi-obstacle (K > 1) step kernels
# The whole library's report: hipcc ... -Rpass-analysis=kernel-resource-usage.
# Usage: bash scripts/regcheck.sh [N] [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
N=${1:-1}; shift || true
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -std=c++17 -mllvm -disable-machine-licm \
  -Iinclude -Iast_sac_amd/csrc -DSHIPSIM_REGCHECK=$N -Rpass-analysis=kernel-resource-usage "$@" \
  ast_sac_amd/csrc/shipsim_kernels.hip -o /tmp/regcheck.so 2> /tmp/regcheck.txt
python3 scripts/regsummary.py /tmp/regcheck.txt | grep -E "ast_step|sbmpc_eval|legacy"
