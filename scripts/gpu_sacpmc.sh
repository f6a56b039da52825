# SQ counters of the SAC kernels (sac_prof.py workload), one pass; prints per-kernel per-wave averages
set -u
TAG=${1:-a}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-include-regex "sac_" --output-format csv -d /tmp/sacpmc_$TAG -o run -- python3 $R/scripts/sac_prof.py > $O/sacpmc_$TAG.log 2>&1; rc=$?
python3 - /tmp/sacpmc_$TAG <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES": n[k] += 1
for k, d in agg.items():
    w = d["SQ_WAVES"] or 1
    print(k, "launches", n[k], {c: round(v / w, 1) for c, v in sorted(d.items())})
PY
exit $rc
