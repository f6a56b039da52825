"""SAC-only workload for rocprofv3: hip-backend FusedSACTrainer, 200 graph-replayed grad steps."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import bench  # noqa: E402

print(bench.bench_sac(torch.device("cuda", 0), 1, None, 200, 256, eager_steps=0))
