"""Per-env-tick instruction inventory of the headline stream (C3: sbmpc, 4096 envs, 4096-tick launches with the
1024-tick launch tail, the bench's action table), for rocprofv3 --pmc passes:
    SHIPSIM_LIB=ast_sac_amd/lib/abl/NAME.so rocprofv3 --pmc ... -- python scripts/tick_inventory.py run OUT.json
writes the env-ticks of every ast_step_kernel dispatch (warmup included) to OUT.json; then
    python scripts/tick_inventory.py summarize PMC_DIR TICKS.json [PMC_DIR TICKS.json ...]
prints SQ counters per env-tick per variant (the ablation builds of scripts/build_variant.sh: differences between
them attribute instructions and cycles to the tick's phases)."""
import collections
import csv
import glob
import json
import os
import sys


def run(out, launches=3):
    import numpy as np
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from ast_sac_amd import shipsim_abi as abi
    from ast_sac_amd.shipsim import ShipSim
    N = 4096
    cfg = abi.ast_config("sbmpc")
    sim = ShipSim(cfg, N)
    sim.reset()
    sim.set_stream_tail(1024)
    n_dec = cfg.max_sampling_frequency
    a_norm = np.random.Generator(np.random.PCG64(20251015)).uniform(-1, 1, (8, n_dec, N)).astype(np.float32)
    table = torch.from_numpy(abi.normalized_to_scoping(a_norm)).cuda()
    ep = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec = torch.zeros(N, dtype=torch.int32, device="cuda")
    ticks = []
    for _ in range(1 + launches):
        o = sim.run_table(table, 4096, ep, dec)
        ticks.append(int(o["ticks"].sum()))
    torch.cuda.synchronize()
    json.dump({"ticks": ticks, "lib": os.environ.get("SHIPSIM_LIB", "in-tree")}, open(out, "w"))
    print(ticks)


def summarize(pairs):
    rows = {}
    for d, tf in zip(pairs[::2], pairs[1::2]):
        ticks = json.load(open(tf))["ticks"]
        tot = collections.defaultdict(float)
        n = 0
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            seen = set()
            for r in csv.DictReader(open(f)):
                if "ast_step_kernel" in r["Kernel_Name"]:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"])
                    seen.add(r["Dispatch_Id"])
            n += len(seen)
        name = os.path.basename(d.rstrip("/"))
        rows[name] = {"dispatches": n, "env_ticks": sum(ticks),
                      **{k: v / sum(ticks) for k, v in sorted(tot.items()) if k != "SQ_WAVES"}}
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        summarize(sys.argv[2:])
