"""Phase split of sac_rows_g4_kernel (block 0, shader clocks) from the timing build
(scripts/build_timing.sh -> ast_sac_amd/lib/abl/libsac_TIMING.so). Diagnostics only."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SACFUSED_LIB"] = os.path.join(ROOT, "ast_sac_amd", "lib", "abl", "libsac_TIMING.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from ast_sac_amd import sacfused  # noqa: E402

print(bench.bench_sac(torch.device("cuda", 0), 1, None, 50, 256, eager_steps=0))
L = sacfused.load_library()
buf = (ctypes.c_ulonglong * 16)()
L.sacf_debug_stamps(buf)
t = [buf[i] for i in range(12)]
names = ["gather", "actor L1", "actor L2", "actor heads+tanh", "critic L1", "critic L2 (x4)", "heads+losses",
         "dg2", "critic bwd + actor scalar", "actor dh2", "actor bwd mv"]
tot = t[11] - t[0]
for k in range(1, 12):
    print(f"{names[k - 1]:>20s} {t[k] - t[k - 1]:8d} cyc {100.0 * (t[k] - t[k - 1]) / tot:5.1f} %")
print("total", tot, "cycles")
