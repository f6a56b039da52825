set -u
TAG=${1:-r1e}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
hard() { rc=$1; if [ $rc -ne 0 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
for ca in none sbmpc; do for lpe in 16 8; do
SHIPSIM_LIB=$R/ast_sac_amd/lib/abl/lib_TIMING.so timeout -k 10 200 python scripts/phase_timing.py $ca $lpe > $O/phase_${TAG}_${ca}_$lpe.log 2>&1; hard $? phase
grep -v amdgpu.ids $O/phase_${TAG}_${ca}_$lpe.log
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sac_$TAG -o run -- python3 $R/scripts/sac_prof.py > $O/prof_sac_$TAG.log 2>&1; hard $? prof_sac
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_env_$TAG -o run -- python3 $R/bench.py --steps 20 --warmup 4 --no-cpu-baseline --sac-steps 0 > $O/prof_env_$TAG.log 2>&1; hard $? prof_env
echo DONE
