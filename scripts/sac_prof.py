"""SAC-only workload for rocprofv3: hip-backend FusedSACTrainer, 200 graph-replayed grad steps."""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

print(bench.bench_sac(torch.device("cuda", 0), 1, None, 200, 256, eager_steps=0))
