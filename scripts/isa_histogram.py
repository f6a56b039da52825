"""Static instruction-class histogram of one kernel's ISA (the file scripts/isa_kernel.sh writes, /tmp/rc/head.s by
default): counts per mnemonic class — FP64 arithmetic, moves (v_mov incl. DPP; s_mov of constant halves), selects,
compares, 32-bit integer, exec-mask logic, branches, waits, lane exchanges, memory.  Static counts weigh every
instruction once, hot or cold; the dynamic class totals come from the PMC passes (scripts/pmc_classes.py).

    python scripts/isa_histogram.py [head.s] [OUT.json]
"""
import collections
import json
import sys


def cls(m):
    if m.startswith("s_"):
        if m.startswith(("s_mov", "s_movk", "s_cmov")):
            return "S_mov (constant halves, addresses)"
        if m.startswith(("s_cbranch", "s_branch")):
            return "S_branch"
        if m.startswith("s_waitcnt"):
            return "S_waitcnt"
        if m.startswith(("s_and", "s_or", "s_xor", "s_andn", "s_orn", "s_not", "s_nand", "s_nor")):
            return "S_logic (exec masks)"
        if m.startswith(("s_load", "s_buffer")):
            return "S_load"
        if m.startswith("s_nop"):
            return "S_nop"
        return "S_other (int, cmp, bfe)"
    if m.startswith("v_"):
        if m.startswith(("v_cmp", "v_cmpx")):
            return "V_cmp"
        if m.startswith("v_cndmask"):
            return "V_cndmask"
        if m.startswith("v_mov") and "dpp" in m:
            return "V_mov_dpp"
        if m.startswith("v_mov"):
            return "V_mov"
        if m.startswith(("v_permlane", "v_readlane", "v_writelane", "v_readfirstlane")):
            return "V_lane xfer"
        if m.startswith("v_accvgpr"):
            return "V_accvgpr"
        if m.startswith("v_cvt"):
            return "V_cvt"
        if "_f64" in m and m.startswith(("v_fma", "v_fmac", "v_add", "v_mul", "v_max", "v_min")):
            return "V_f64 fma/add/mul/minmax"
        if "_f64" in m and m.startswith(("v_rcp", "v_sqrt", "v_rsq", "v_div", "v_ldexp", "v_frexp", "v_fract",
                                         "v_floor", "v_trig", "v_ceil", "v_rndne", "v_trunc")):
            return "V_f64 other (rcp, div steps, ldexp, frexp)"
        if "_f32" in m:
            return "V_f32"
        return "V_int32 / bit ops"
    if m.startswith("ds_"):
        return "LDS"
    if m.startswith(("global_", "buffer_", "flat_")):
        return "VMEM"
    return "other"


def main(path="/tmp/rc/head.s", out=None):
    L = open(path).read().split("\n")
    ins = [l.strip().split()[0] for l in L if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    per = collections.Counter(ins)
    k = collections.Counter()
    for m, n in per.items():
        k[cls(m)] += n
    tot = sum(k.values())
    res = dict(instructions=tot, classes={a: b for a, b in k.most_common()},
               share={a: round(b / tot, 4) for a, b in k.most_common()}, top_mnemonics=per.most_common(40))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
    for a, b in k.most_common():
        print(f"{a:44s} {b:6d} {100 * b / tot:5.1f}%")
    print("total", tot)


if __name__ == "__main__":
    main(*sys.argv[1:])
