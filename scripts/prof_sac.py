"""SAC grad steps alone (runner networks 2x256, batch 256, replay sampling on the device), for
`rocprofv3 --kernel-trace --stats -- python scripts/prof_sac.py`: per-kernel durations of one step."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--graph", type=int, default=0)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    r = bench.bench_sac(dev, 1, None, a.steps, a.batch, eager_steps=0, graph=bool(a.graph))
    print({k: v for k, v in r.items() if k != "impl"})


if __name__ == "__main__":
    main()
