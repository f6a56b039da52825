"""FP64 VALU counters of ast_step_kernel from one rocprofv3 --pmc pass (SQ block, 8 counters):
SQ_INSTS_VALU_FLOPS_FP64, SQ_INSTS_VALU_FLOPS_FP64_TRANS, SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F64,
SQ_INSTS_VALU, SQ_WAVES. Writes a per-launch record read by bench.py (roofline.fp64_valu).

    python scripts/pmc_fp64.py gpurun_out/pmc_fp64_TAG profiles/round2_pmc_fp64.json collav envs slice
"""
import collections
import csv
import glob
import json
import os
import sys

COUNTERS = ("SQ_INSTS_VALU_FLOPS_FP64", "SQ_INSTS_VALU_FLOPS_FP64_TRANS", "SQ_INSTS_VALU_FMA_F64",
            "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU", "SQ_WAVES")


def main(d, out, collav="sbmpc", envs="4096", slice_ticks="4096"):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "ast_step_kernel" in r["Kernel_Name"] and r["Counter_Name"] in COUNTERS:
                per[(f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    n = len(per)
    avg = {c: sum(v[c] for v in per.values()) / n for c in COUNTERS}
    res = dict(kernel="ast_step_kernel", collav=collav, envs=int(envs), slice=int(slice_ticks), dispatches=n,
               per_launch=avg,
               # SQ_INSTS_VALU_FLOPS_FP64 = 2 FMA + ADD + MUL + TRANS wave-instructions (it equals that sum of the
               # instruction counters exactly), so the lane FLOPs a wave issues are 64x it
               fp64_flops_per_launch=64.0 * avg["SQ_INSTS_VALU_FLOPS_FP64"],
               fp64_wave_instructions_per_launch=(avg["SQ_INSTS_VALU_FMA_F64"] + avg["SQ_INSTS_VALU_ADD_F64"]
                                                  + avg["SQ_INSTS_VALU_MUL_F64"] + avg["SQ_INSTS_VALU_TRANS_F64"]),
               note="one rocprofv3 --pmc pass of python3 bench.py --no-cpu-baseline --sac-steps 0 --no-c2 "
                    "(default steps/warmup), averaged over every ast_step_kernel dispatch; fp64_flops_per_launch = 64 lanes x "
                    "SQ_INSTS_VALU_FLOPS_FP64 (issued lane-FLOPs: exec-masked lanes included)")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:])
