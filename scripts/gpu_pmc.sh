# SQ counters for ast_step_kernel + SAC kernels (separate --pmc passes), SAC timing variants
set -u
TAG=${1:-pmc}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
timeout -k 10 600 python -m pytest tests/test_sac.py -m gpu -q -p no:cacheprovider -x > $O/pytest_sac_$TAG.log 2>&1; ok $? pytest
tail -3 $O/pytest_sac_$TAG.log
for rows in 4x1 2x2 2x4 1x4; do
  SACF_ROWS=$rows timeout -k 10 200 python scripts/sac_prof.py > $O/sac_rows_${TAG}_$rows.log 2>&1; hard $? sac_$rows
  echo "rows $rows: $(tail -1 $O/sac_rows_${TAG}_$rows.log | cut -c1-80)"
done
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $O/pmc_sq${i}_$TAG -o run -- python3 $R/bench.py --steps 10 --warmup 4 --no-cpu-baseline --sac-steps 0 > $O/pmc_sq${i}_$TAG.log 2>&1; ok $? pmc_$i
done
echo DONE
