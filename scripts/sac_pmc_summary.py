"""Per-kernel means of the SAC PMC passes (scripts/gpu/sac_pmc.sh): FETCH_SIZE ×2 (gfx950 reports half the bytes of
wide reads, MI355X_MICROARCH.md HBM section) and WRITE_SIZE in bytes per dispatch, L2 hit rate, L1 requests.
    python scripts/sac_pmc_summary.py gpurun_out/pmc_sac_TAG N_PASSES > out.json"""
import collections
import csv
import glob
import json
import re
import sys


def main(prefix, n):
    res = collections.defaultdict(lambda: collections.defaultdict(list))
    for i in range(int(n)):
        per = collections.defaultdict(float)
        name = {}
        for f in glob.glob(f"{prefix}_{i}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if "sac_" not in k:
                    continue
                m = re.search(r"(sac_\w+?_kernel)", k)
                kk = m.group(1) if m else k[:40]
                per[(kk, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
                name[kk] = k
        for (kk, _, c), v in per.items():
            res[kk][c].append(v)
    out = {}
    for kk, cs in res.items():
        o = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"dispatches": max(len(v) for v in cs.values())}
        if "FETCH_SIZE" in o:
            d["fetch_bytes"] = 2 * 1024 * o["FETCH_SIZE"]
        if "WRITE_SIZE" in o:
            d["write_bytes"] = 1024 * o["WRITE_SIZE"]
        if "TCC_HIT_sum" in o:
            d["l2_hit_rate"] = o["TCC_HIT_sum"] / max(1.0, o["TCC_HIT_sum"] + o["TCC_MISS_sum"])
            d["l2_requests"] = o["TCC_HIT_sum"] + o["TCC_MISS_sum"]
        for c in ("TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum"):
            if c in o:
                d[c] = o[c]
        out[kk] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
