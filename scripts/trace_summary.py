"""Summarise a rocprofv3 kernel trace of the default bench command (ast_step_kernel launches) next to
the bench's own HIP-event numbers; writes a small JSON and deletes the (large) trace CSV.
Usage: python scripts/trace_summary.py <rocprof out dir> <bench log> <out.json>"""
import csv
import glob
import json
import os
import re
import sys

# the decision-stream (CHAIN 1, shipsim_run_table) instantiation of two-ship envs (SLOTS 2) the headline times; the
# bench's secondary lines run other instantiations: the policy stream (CHAIN 2), the C4 shard (LPE 8) and the C5
# multi-obstacle legs (SLOTS 4 / 8)
TABLE = re.compile(r"ast_step_kernel<true,\s*\d+,\s*16,\s*false,\s*1,\s*2>")

d, bench_log, out = sys.argv[1:4]
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if TABLE.search(r["Kernel_Name"]):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    os.remove(f)
rows.sort()
ms = [x[1] / 1e6 for x in rows]
line = [ln for ln in open(bench_log) if ln.startswith("{")][-1]
b = json.loads(line)
res = dict(command="rocprofv3 --kernel-trace --stats -- python3 bench.py (default bench command)",
           ast_step_kernel_dispatches=len(ms), mean_ms_all=sum(ms) / max(1, len(ms)),
           mean_ms_timed_last=sum(ms[-b["steps"]:]) / max(1, len(ms[-b["steps"]:])),
           bench_kernel_ms_all_launches=b["roofline"].get("kernel_ms_all_launches"),
           bench_kernel_ms_timed=b["roofline"].get("kernel_ms_timed"))
for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):  # rocprof's own per-kernel means
    for r in csv.DictReader(open(f)):
        if TABLE.search(r["Name"]):
            res["stats_kernel"] = r["Name"]
            res["stats_calls"] = int(r["Calls"])
            res["stats_mean_ms"] = float(r["AverageNs"]) / 1e6
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
