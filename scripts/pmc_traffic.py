"""HBM traffic of ast_step_kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; KB).

Per MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE reports half the bytes of wide reads on gfx950
-> x2; WRITE_SIZE is taken as is. Writes profiles/<tag>_pmc_traffic.json, read by bench.py.

    python scripts/pmc_traffic.py gpurun_out/pmc_fetch_r1a gpurun_out/pmc_write_r1a profiles/round1_pmc_traffic.json
"""
import collections
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kernel="ast_step_kernel"):
    vals = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    return list(vals.values())


def main(fetch_dir, write_dir, out, slice_ticks="4096", collav="sbmpc", envs=4096):
    fe = per_dispatch(fetch_dir, "FETCH_SIZE")
    wr = per_dispatch(write_dir, "WRITE_SIZE")
    fetch_b = 2 * 1024 * sum(fe) / len(fe)
    write_b = 1024 * sum(wr) / len(wr)
    res = dict(kernel="ast_step_kernel", collav=collav, envs=envs, slice=int(slice_ticks), dispatches=[len(fe), len(wr)],
               fetch_size_kb_raw=sum(fe) / len(fe), write_size_kb=sum(wr) / len(wr),
               fetch_bytes_corrected=fetch_b, write_bytes=write_b, hbm_bytes_per_launch=fetch_b + write_b,
               note="FETCH_SIZE x2 (gfx950 wide-read correction, MI355X_MICROARCH.md HBM section); "
                    "python3 bench.py --no-cpu-baseline --sac-steps 0 (default steps/warmup/slice), averaged over "
                    "every ast_step_kernel dispatch of the run")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:5])
