# Per-launch durations of the weight-gradient pass split in two (SACF_WG_MODE=1): MFMA tiles vs the rest.
set -u
TAG=${1:-wg3}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
for m in 1 0; do
SACF_WG_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_wg${m}_$TAG -o run -- python scripts/prof_sac.py --steps 300 --graph 1 > $O/wgtrace${m}_$TAG.log 2>&1 || { echo STOP prof; exit 3; }
f=$(find $O/trace_wg${m}_$TAG -name '*kernel_trace.csv' | head -1)
python - "$f" $m <<'PY'
import csv, sys, collections, statistics
rows = list(csv.DictReader(open(sys.argv[1])))
print("columns:", [c for c in rows[0].keys()][:30]) if sys.argv[2] == "1" else None
d = collections.defaultdict(list)
for r in rows:
    if "sac_" not in r["Kernel_Name"]:
        continue
    g = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
    d[(r["Kernel_Name"][22:52], g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items()):
    print("mode", sys.argv[2], k, len(v), "median ns", statistics.median(v))
PY
done
find $O -name "*kernel_trace.csv" -delete
