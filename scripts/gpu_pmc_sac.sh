# SQ counters of the SAC kernels (instruction-fetch vs memory waits). Usage: bash scripts/gpu_pmc_sac.sh TAG
set -u
TAG=${1:-sacpmc}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_IFETCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d $O/pmc_$TAG -o run -- python3 $R/scripts/prof_sac.py --steps 200 --graph 1 > $O/pmc_$TAG.log 2>&1 || { echo STOP; tail -5 $O/pmc_$TAG.log; exit 3; }
cd $R
python - <<PY
import csv, glob, collections
f = glob.glob("$O/pmc_$TAG/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "sac_" not in k: continue
    k = k.split("(")[0].split("::")[-1][:28]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    c = {m: v / n[(k, m)] for m, v in d.items()}
    w = c.get("SQ_WAVE_CYCLES", 1)
    print(k.ljust(28), "waves %5.0f" % c.get("SQ_WAVES", 0), "wave_cyc/wave %7.0f" % (w / max(c.get("SQ_WAVES", 1), 1)),
          "wait_inst %.2f" % (c.get("SQ_WAIT_INST_ANY", 0) / w), "wait_any %.2f" % (c.get("SQ_WAIT_ANY", 0) / w),
          "active %.2f" % (c.get("SQ_ACTIVE_INST_ANY", 0) / w), "ifetch/wave %.0f" % (c.get("SQ_IFETCH", 0) / max(c.get("SQ_WAVES", 1), 1)),
          "valu/wave %.0f" % (c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_WAVES", 1), 1)), "salu/wave %.0f" % (c.get("SQ_INSTS_SALU", 0) / max(c.get("SQ_WAVES", 1), 1)))
PY
