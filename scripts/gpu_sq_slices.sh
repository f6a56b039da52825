# SQ counters of the default sbmpc bench kernel at 128- and 2048-tick launches (wave occupancy of the
# launch = SQ_WAVE_CYCLES / (waves x launch cycles): the slowest-wave tail).
set -u
TAG=${1:-sq}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
cd /tmp && export TMPDIR=/tmp
for cfg in "128 16 12" "2048 3 1"; do
  set -- $cfg
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/sq_${TAG}_$1 -o run -- python3 $R/bench.py --slice $1 --steps $2 --warmup $3 --no-cpu-baseline --sac-steps 0 --no-c2 > $O/sq_${TAG}_$1.log 2>&1; hard $? sq_$1
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O/kt_${TAG}_$1 -o run -- python3 $R/bench.py --slice $1 --steps $2 --warmup $3 --no-cpu-baseline --sac-steps 0 --no-c2 > $O/kt_${TAG}_$1.log 2>&1; hard $? kt_$1
done
echo DONE
