"""Per-request cost of the device SBMPC optimisers (shipsim_sbmpc_eval, shipsim_sbmpc_eval_multi): the same random
requests (half of the obstacles on a collision course, as tests/test_gpu_sbmpc_multi.py draws them) served densely
(every lane of a wave requests: two requests per pass) and sparsely (one request per wave: the lone-request pass),
for the single-obstacle service and the multi-obstacle one at K = 1, 2, 4.  Prints one JSON line (µs per launch,
ns per request).  Usage: python scripts/sbmpc_bench.py [n]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ast_sac_amd import shipsim_abi as abi  # noqa: E402
from ast_sac_amd.shipsim import sbmpc_eval, sbmpc_eval_multi  # noqa: E402
from test_gpu_sbmpc_multi import _random_requests  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    rng = np.random.Generator(np.random.PCG64(3))
    res = {"n": n}
    for K in (1, 2, 4):
        req = _random_requests(rng, n, K)
        sparse = req.copy()
        far = np.ones(n, bool)
        far[::64] = False
        for k in range(abi.MAX_OBS):
            sparse[far, 10 + 7 * k] += 1e5
        for name, r in (("dense", req), ("lone", sparse)):
            x = torch.as_tensor(r, device="cuda")
            active = int(sbmpc_eval_multi(x, K)[:, 2].sum().item())
            t = timed(lambda: sbmpc_eval_multi(x, K))
            res[f"multi_k{K}_{name}"] = {"us": t * 1e6, "active": active, "ns_per_active": t * 1e9 / max(active, 1)}
            if K == 1:
                single = torch.as_tensor(np.concatenate([r[:, :10], r[:, 10:15], r[:, 15:17]], 1), device="cuda")
                t = timed(lambda: sbmpc_eval(single))
                res[f"single_{name}"] = {"us": t * 1e6, "active": active, "ns_per_active": t * 1e9 / max(active, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
