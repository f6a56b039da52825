# Assembly of one ast_step_kernel instantiation from a narrowed build, to /tmp/rc/head.s.
# Usage: bash scripts/isa_kernel.sh MANGLED_PREFIX [extra hipcc flags, e.g. -DSHIPSIM_REGCHECK=2]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p /tmp/rc && cd /tmp/rc
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -std=c++17 -I$R/include -I$R/ast_sac_amd/csrc \
  -mllvm -disable-machine-licm -mllvm -amdgpu-sched-strategy=max-ilp -mllvm -amdgpu-use-amdgpu-trackers --save-temps "${@:2}" $R/ast_sac_amd/csrc/shipsim_kernels.hip -o /tmp/rc/x.so 2>/dev/null
python3 - "$1" <<'PY'
import sys
L = open('/tmp/rc/shipsim_kernels-hip-amdgcn-amd-amdhsa-gfx950.s').read().split('\n')
st = [i for i, l in enumerate(L) if l.startswith(sys.argv[1]) and ':' in l][0]
en = [i for i in range(st, len(L)) if L[i].startswith('.Lfunc_end')][0]
open('/tmp/rc/head.s', 'w').write('\n'.join(L[st:en]))
ins = [l for l in L[st:en] if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
print(len(ins), 'instructions;', sum('v_writelane' in l for l in ins), 'writelane;', sum('v_readlane' in l for l in ins), 'readlane;',
      sum('accvgpr' in l for l in ins), 'accvgpr moves')
PY
