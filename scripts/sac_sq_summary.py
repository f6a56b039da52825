"""Summarise the SAC SQ counter pass (scripts/gpu/round.sh, sac.sh: rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES
SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA over scripts/prof_sac.py):
per-dispatch means per kernel, per-wave cycles (the quad-cycle counters x4) and their shares.
Usage: python scripts/sac_sq_summary.py DIR TAG > out.json"""
import collections
import csv
import glob
import json
import os
import re
import sys

d, tag = sys.argv[1], sys.argv[2]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0]
        per[(name, f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
by = collections.defaultdict(list)
for (name, _, _), v in per.items():
    by[name].append(v)
out = {}
for name, rows in sorted(by.items()):
    keys = sorted({k for v in rows for k in v})
    avg = {k: sum(v.get(k, 0.0) for v in rows) / len(rows) for k in keys}
    waves = max(avg.get("SQ_WAVES", 0.0), 1.0)
    cyc = {k: avg[k] * 4 / waves for k in ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")
           if k in avg}
    # SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_ANY count quad-cycles (x4); SQ_BUSY_CYCLES is per SE
    tot = cyc.get("SQ_WAVE_CYCLES", 1.0)
    out[name] = dict(avg, dispatches=len(rows), per_wave_cycles=cyc,
                     share_of_wave_cycles={k: v / tot for k, v in cyc.items() if k != "SQ_WAVE_CYCLES"},
                     valu_per_wave=avg.get("SQ_INSTS_VALU", 0.0) / waves, mfma_per_wave=avg.get("SQ_INSTS_MFMA", 0.0) / waves)
print(json.dumps({"command": "rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
                  "SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA -- python3 scripts/prof_sac.py --steps 200 --graph 1 "
                  f"(B=256, 2x256; {tag})", "note": "per dispatch means; quad-cycle counters x4 = cycles; WAIT_ANY = "
                  "parked on s_waitcnt / barrier, WAIT_INST_ANY = issue stall", "per_dispatch_mean": out}, indent=1))
