"""Whole-library register report: recompile libshipsim and libsacfused with the build's exact flags plus
-Rpass-analysis=kernel-resource-usage (into /tmp, the in-tree libraries are untouched) and print one line per
kernel (VGPR / AGPR / SGPR, spills, scratch, occupancy), then the kernels that spill.
Usage: python scripts/register_report.py > profiles/<round>/register_usage.txt   """
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import HIPCC, HIPFLAGS, SAC_SRC, SRC  # noqa: E402
from ast_sac_amd.build_hash import lib_flag_sets  # noqa: E402


def report(name, src):
    err = ""
    for i, flags in enumerate(lib_flag_sets(name)):  # every object of the library with its own flags
        cmd = [HIPCC] + HIPFLAGS + flags + ["-Rpass-analysis=kernel-resource-usage"] + src + \
            ["-o", f"/tmp/regreport_{name}_{i}.so"]
        err += subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
    rows, cur = {}, None
    for line in err.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+): (\d+)", line)
        if m and cur:
            rows[cur][m.group(1).strip()] = int(m.group(2))
    names = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.splitlines()
    out = []
    for (k, v), dn in zip(rows.items(), names):
        out.append((dn, v))
    return out


def main():
    spill = []
    total = 0
    for name, src in (("shipsim", SRC), ("sacfused", SAC_SRC)):
        print(f"== lib{name}.so ==")
        for dn, v in report(name, src):
            total += 1
            s, vs = v.get("SGPRs Spill", 0), v.get("VGPRs Spill", 0)
            print(f"{dn}\n    VGPR {v.get('VGPRs')} AGPR {v.get('AGPRs')} SGPR {v.get('TotalSGPRs')} sgpr_spill {s} "
                  f"vgpr_spill {vs} scratch {v.get('ScratchSize [bytes/lane]')} occ {v.get('Occupancy [waves/SIMD]')} lds {v.get('LDS Size [bytes/block]')}")
            if s or vs:
                spill.append((name, dn, s, vs))
    print(f"\n== {total} kernels, {len(spill)} with spills ==")
    for name, dn, s, vs in spill:
        print(f"lib{name}: sgpr_spill {s} vgpr_spill {vs}  {dn}")


if __name__ == "__main__":
    main()
