# Register usage / spills of the headline step kernels (chained, LPE 16, detailed; sbmpc and none) from a
# narrowed build (-DSHIPSIM_REGCHECK instantiates only those). Usage: bash scripts/regcheck.sh [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -std=c++17 -Iinclude -Iast_sac_amd/csrc \
  -DSHIPSIM_REGCHECK -Rpass-analysis=kernel-resource-usage "$@" ast_sac_amd/csrc/shipsim_kernels.hip -o /tmp/regcheck.so 2> /tmp/regcheck.txt
python3 scripts/regsummary.py /tmp/regcheck.txt | grep -E "ast_step|sbmpc_eval"
