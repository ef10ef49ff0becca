"""Summarise rocprofv3 --pmc passes of the bench into the roofline's traffic
and VALU figures for the dominant kernel (k_bucket_acc_chunk) at the bench's
grid size.  gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE
reports half of the bytes of wide coalesced reads -> x2; WRITE_SIZE as is.
FETCH/WRITE_SIZE are in KB (rocprofv3 derived metrics, 1024 B).

    python tools/pmc_summary.py OUT.json DIR_FETCH DIR_WRITE DIR_VALU
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter, match="k_bucket_acc_short"):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and match in r["Kernel_Name"]:
                vals[int(r["Grid_Size"])].append(float(r["Counter_Value"]))
    return vals


def main():
    out, dfetch, dwrite, dvalu = sys.argv[1:5]
    fetch = load(dfetch, "FETCH_SIZE")
    write = load(dwrite, "WRITE_SIZE")
    valu = load(dvalu, "SQ_INSTS_VALU")
    grid = max(fetch, key=lambda g: len(fetch[g]))  # the bench's launches dominate the count
    avg = lambda v: sum(v) / len(v)  # noqa: E731
    f_kb, w_kb = avg(fetch[grid]), avg(write.get(grid, [0.0]))
    res = {
        "kernel": "k_bucket_acc_short<Fq> (bench: 2^20-point G1 MSM, GLV, c = 16)",
        "grid": grid, "launches": {"fetch": len(fetch[grid]), "write": len(write.get(grid, [])),
                                   "valu": len(valu.get(grid, []))},
        "fetch_size_kb_per_launch": f_kb, "write_size_kb_per_launch": w_kb,
        "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE as reported; KB = 1024 B",
        "hbm_bytes_per_launch": (2 * f_kb + w_kb) * 1024.0,
        "valu_insts_per_launch": avg(valu[grid]) if valu.get(grid) else None,
        "other_grids": {str(g): len(v) for g, v in fetch.items() if g != grid},
        "note": "FETCH counts fabric requests incl. Infinity-Cache hits: bases gathered once per window entry",
    }
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
