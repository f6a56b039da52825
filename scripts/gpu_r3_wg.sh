# SAC weight-gradient launch modes (SACF_WG_MODE 0 one launch / 1 MFMA tiles then the rest / 2 rest first):
# grad-step rate, then rocprofv3 kernel stats of modes 0 and 1. Usage: bash scripts/gpu_r3_wg.sh TAG
set -u
TAG=${1:-wg}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
SACF_WG_MODE=1 timeout -k 10 300 python -u -m pytest tests/test_sac.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$TAG.log 2>&1
rc=$?; tail -2 $O/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for m in 0 1 2; do for b in 64 256; do
  echo "mode $m B $b: $(SACF_WG_MODE=$m timeout -k 10 120 python scripts/prof_sac.py --steps 3000 --graph 1 --batch $b 2>&1 | tail -1 | cut -c1-100)"
done; done; done
export TMPDIR=/tmp
for m in 0 1; do
  SACF_WG_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_wg${m}_$TAG -o run -- python scripts/prof_sac.py --steps 300 --graph 1 > $O/wgprof${m}_$TAG.log 2>&1 || { echo STOP prof; exit 3; }
  f=$(find $O/prof_wg${m}_$TAG -name '*kernel_stats.csv' | head -1)
  python -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'sac_' in r['Name']: print('mode $m', r['Name'][22:60].ljust(40), r['Calls'], r['AverageNs'])
"
done
find $O -name "*kernel_trace.csv" -delete
