"""Instruction-class inventory per env-tick of the headline kernel (ast_step_kernel, the bench's C3 stream), from
rocprofv3 --pmc passes of the same bench command (scripts/gpu/inventory_classes.sh), each pass at most 8 SQ counters.
The VALU classes the SQ block counts (INT32, INT64, CVT, FMA / ADD / MUL / TRANS in F32 and F64) and the remainder
of SQ_INSTS_VALU they leave: register moves (v_mov, constants into VGPRs), selects (v_cndmask), compares, DPP /
permlane / readlane exchanges, bit operations on f64 halves (ldexp, frexp, class) — the kinds the static histogram
of the kernel's ISA (scripts/isa_histogram.py) splits further. Env-ticks per launch come from the bench line of the
same run.

    python scripts/pmc_classes.py OUT.json BENCH.json DIR1 [DIR2 ...]
"""
import collections
import csv
import glob
import json
import os
import sys


def main(out, bench_json, *dirs):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "ast_step_kernel" in r["Kernel_Name"]:
                    per[(d, f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    tot = collections.defaultdict(list)
    for v in per.values():
        for c, x in v.items():
            tot[c].append(x)
    avg = {c: sum(x) / len(x) for c, x in tot.items()}
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    ticks = b["value"] * b["ms_per_step"] * 1e-3  # env-ticks per launch
    pt = {c: v / ticks for c, v in avg.items()}
    valu = pt.get("SQ_INSTS_VALU", float("nan"))
    known = sum(pt.get(c, 0.0) for c in ("SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT",
                                           "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                           "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32",
                                           "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32"))
    res = dict(kernel="ast_step_kernel (bench C3 stream)", env_ticks_per_launch=ticks, dispatches=len(per),
               per_env_tick=pt, valu_per_env_tick=valu,
               valu_unclassified_per_env_tick=valu - known,
               note="wave-instructions per env-tick (a wave holds 64 / lanes_per_env envs); 'unclassified' = VALU "
                    "minus the SQ block's INT32 / INT64 / CVT / F32 / F64 classes: moves, selects, compares, "
                    "lane exchanges, f64 bit operations")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:])
