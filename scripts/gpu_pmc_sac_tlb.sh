# TLB / L2 counters of the SAC kernels (diagnostics). Usage: bash scripts/gpu_pmc_sac_tlb.sh TAG
set -u
TAG=${1:-tlb}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_REQUEST_sum TCC_HIT_sum TCC_MISS_sum SQ_WAVES --output-format csv -d $O/pmc_$TAG -o run -- python3 $R/scripts/prof_sac.py --steps 200 --graph 1 > $O/pmc_$TAG.log 2>&1 || { echo STOP; tail -3 $O/pmc_$TAG.log; exit 3; }
echo done
