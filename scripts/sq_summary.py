"""Summarise SQ counter passes of ast_step_kernel: per-wave cycles split into instruction-fetch waits,
any-wait and issue, VALU per wave. Usage: python scripts/sq_summary.py DIR [DIR...]"""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "ast_step_kernel" in r["Kernel_Name"]:
                per[(f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        print(d, "no ast_step_kernel dispatches")
        continue
    keys = sorted({k for v in per.values() for k in v})
    avg = {k: sum(v.get(k, 0.0) for v in per.values()) / len(per) for k in keys}
    w = avg.get("SQ_WAVE_CYCLES", 1.0)
    waves = max(avg.get("SQ_WAVES", 1.0), 1.0)
    print(os.path.basename(d.rstrip("/")), "dispatches", len(per))
    for k in keys:
        print(f"  {k:24s} {avg[k]:16.4g}   per wave {avg[k] / waves:14.6g}   frac of wave cycles {avg[k] / w:8.4f}")
