"""SAC step timing probe: FusedSACTrainer graph vs eager, hipBLASLt vs rocBLAS backends."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
for lib in ("cublaslt", "cublas"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:  # noqa: BLE001
        print(lib, "unavailable", e)
        continue
    r = bench.bench_sac(dev, 1, None, 300, 256, eager_steps=40)
    print(lib, {k: v for k, v in r.items() if k != "impl"}, flush=True)
