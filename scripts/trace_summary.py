"""Summarise a rocprofv3 kernel trace of the default bench command (ast_step_kernel launches) next to
the bench's own HIP-event numbers; writes a small JSON and deletes the (large) trace CSV.
Usage: python scripts/trace_summary.py <rocprof out dir> <bench log> <out.json>"""
import csv
import glob
import json
import os
import re
import sys

# the decision-stream (CHAIN 1, shipsim_run_table) instantiations the headline times; the bench's secondary
# policy-stream line (CHAIN 2) runs the same kernel template with the policy in the loop
TABLE = re.compile(r"ast_step_kernel<[^>]*,\s*1,\s*\d+>")

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
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
