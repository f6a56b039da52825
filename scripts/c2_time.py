"""C2 (configs[1]) ship-ticks/s alone: bench.bench_c2 on the library SHIPSIM_LIB names (or the in-tree one)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

if __name__ == "__main__":
    per = {30: int(sys.argv[1]), 4: int(sys.argv[2])} if len(sys.argv) > 2 else None
    r = bench.bench_c2(torch.device("cuda", 0), per_launch=per)
    r["per_launch"] = per
    r["lib"] = os.environ.get("SHIPSIM_LIB", "in-tree")
    print(json.dumps(r))
