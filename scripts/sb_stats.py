"""Multi-obstacle SBMPC activity of the C5 decision stream (bench.py's bench_c5 workload), from a diagnostics build
with -DSHIPSIM_SB_STATS (scripts/build_variant.sh NAME -DSHIPSIM_REGCHECK=3 -DSHIPSIM_SB_STATS), run through
SHIPSIM_LIB on the GPU box:  SHIPSIM_LIB=ast_sac_amd/lib/abl/NAME.so python scripts/sb_stats.py K [launches]
Prints one JSON line: per env-tick request rate, passes per optimiser call, lone-request share, horizons per pass."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from ast_sac_amd.shipsim import load_library  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    L = load_library()
    out = (C.c_uint32 * 32)()
    dev = torch.device("cuda", 0)
    L.shipsim_diag_lane_faults(out)  # zero the counters
    r = bench.bench_c5(dev, 1, 4096, K, launches=launches, warmup=0)
    torch.cuda.synchronize()
    assert L.shipsim_diag_lane_faults(out) == 0, "not an SHIPSIM_SB_STATS build"
    v = [out[16 + 2 * i] | (out[17 + 2 * i] << 32) for i in range(8)]
    names = ["wave_ticks_with_pass", "passes", "lone_passes", "requests_served", "horizon_lanes", "far_lanes",
             "env_ticks_requesting", "env_ticks"]
    d = dict(zip(names, v))
    d.update(K=K, env_ticks_per_s=r["env_ticks_per_s"],
             request_rate=v[6] / max(v[7], 1), passes_per_call=v[1] / max(v[0], 1), lone_share=v[2] / max(v[1], 1),
             horizon_lanes_per_pass=v[4] / max(v[1], 1), far_lanes_per_pass=v[5] / max(v[1], 1),
             wave_ticks_with_pass_per_env_tick=v[0] / max(v[7], 1))
    print(json.dumps(d))


if __name__ == "__main__":
    main()
