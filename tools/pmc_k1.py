"""Summarise rocprofv3 --pmc passes of tools/prof_open.py 24 (the 2^24
sqrt-PST commit) for K1's accumulation kernel k_bucket_acc_chunk<Fq> (one
launch per commit): HBM / fabric bytes per launch with the gfx950 FETCH_SIZE
x2 correction (MI355X_MICROARCH.md), VALU instructions per launch, and the
per-launch duration from a kernel trace of the same script.

    python tools/pmc_k1.py OUT.json DIR_FETCH DIR_WRITE DIR_VALU DIR_TRACE
"""
import csv
import glob
import json
import os
import sys

KERNEL = "k_bucket_acc_chunk"


def values(d, counter):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and KERNEL in r["Kernel_Name"]:
                out.append(float(r["Counter_Value"]))
    return out


def main():
    out, dfetch, dwrite, dvalu, dtrace = sys.argv[1:6]
    fetch, write, valu = values(dfetch, "FETCH_SIZE"), values(dwrite, "WRITE_SIZE"), values(dvalu, "SQ_INSTS_VALU")
    avg = lambda v: sum(v) / len(v) if v else None  # noqa: E731
    durs = []
    for f in glob.glob(os.path.join(dtrace, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    rows, npts, W = 4096, 4096, 22  # 2^24: 4096 rows of 4096 scalars, 22 windows of 12 bits
    madds = rows * npts * W          # one table gather + mixed add per (row, point, window) entry
    f_kb, w_kb = avg(fetch), avg(write) or 0.0
    hbm = (2 * f_kb + w_kb) * 1024.0 if f_kb is not None else None
    res = {"kernel": "k_bucket_acc_chunk<Fq> (K1, 2^24 sqrt-PST commit: 4096 rows x 4096 points, c = 12)",
           "launches": len(fetch), "fetch_size_kb_per_launch": f_kb, "write_size_kb_per_launch": w_kb,
           "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE as reported; KB = 1024 B",
           "hbm_bytes_per_launch": hbm, "valu_insts_per_launch": avg(valu),
           "kernel_ms": avg(durs), "table_gathers_per_launch": madds,
           "gather_bytes_per_launch": madds * 96,
           "fabric_bytes_per_gather": hbm / madds if hbm else None,
           "achieved_gather_gbs": (madds * 96 / (avg(durs) * 1e-3) / 1e9) if durs else None,
           "note": "fabric bytes count Infinity-Cache hits too: the 8.65 MB window table is gathered per entry"}
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
