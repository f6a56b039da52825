# rocprofv3 kernel stats of the SAC-only workload (scripts/sac_prof.py); copies the stats CSV only
set -u
TAG=${1:-sp}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O/sacprof_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sacprof_$TAG -o run -- python3 $R/scripts/sac_prof.py > $O/sacprof_$TAG.log 2>&1; rc=$?
find /tmp/sacprof_$TAG -name "*kernel_stats*" -exec cp {} $O/sacprof_$TAG/ \;
python3 - "$O/sacprof_$TAG" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "sac_" in r["Name"]:
            print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us")
PY
tail -1 $O/sacprof_$TAG.log
exit $rc
