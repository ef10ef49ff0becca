"""Summarise rocprofv3 --pmc passes of the bench into the roofline's traffic
and VALU figures for the dominant kernel (k_bucket_acc_short): the MSM runs
one launch per window group (msm.hip msm_groups), so the figures are per MSM
= the sum over one call's launches (launch count of the rarest grid = MSMs).  gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE
reports half of the bytes of wide coalesced reads -> x2; WRITE_SIZE as is.
FETCH/WRITE_SIZE are in KB (rocprofv3 derived metrics, 1024 B).

The VALU pass also holds the bench's Fq-multiply microbenchmark (k_mb_fq29,
the accumulation's radix-2^29 product, 200 per lane; k_mb_fqmul before round 4): its SQ_INSTS_VALU per wave-product against the
accumulation's per wave-madd gives the mixed add's cost in Fq-product
equivalents from counted instructions (bench.py's compute column).  With a
kernel-trace directory of the same bench, the per-grid launch durations of the
accumulation are added, so its per-MSM kernel time can be read from this file.

    python tools/pmc_summary.py OUT.json DIR_FETCH DIR_WRITE DIR_VALU [DIR_TRACE]
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
    dtrace = sys.argv[5] if len(sys.argv) > 5 else None
    fetch = load(dfetch, "FETCH_SIZE")
    write = load(dwrite, "WRITE_SIZE")
    valu = load(dvalu, "SQ_INSTS_VALU")
    mb = load(dvalu, "SQ_INSTS_VALU", "k_mb_fq29")  # the accumulation's product (field29.h, bench MB_FQMUL_KIND)
    if not mb:
        mb = load(dvalu, "SQ_INSTS_VALU", "k_mb_fqmul")
    avg = lambda v: sum(v) / len(v)  # noqa: E731
    n_msm = min(len(v) for v in fetch.values())
    per_msm = lambda d: sum(sum(v) for v in d.values()) / n_msm if d else None  # noqa: E731
    f_kb, w_kb = per_msm(fetch), per_msm(write) or 0.0
    res = {
        "kernel": "k_bucket_acc_short[_lds]<Fq> (bench: 2^20-point G1 MSM, GLV, c = 16, one launch per window group)",
        "grids": {str(g): len(v) for g, v in fetch.items()}, "msm_calls": n_msm,
        "fetch_size_kb_per_msm": f_kb, "write_size_kb_per_msm": w_kb,
        "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE as reported; KB = 1024 B",
        "hbm_bytes_per_launch": (2 * f_kb + w_kb) * 1024.0,
        "hbm_bytes_note": "per MSM (all window-group launches of one call), the unit of bench.py kernel_ms_per_msm",
        "valu_insts_per_launch": per_msm(valu),
        "per_grid_avg_fetch_kb": {str(g): avg(v) for g, v in fetch.items()},
        "note": "FETCH counts fabric requests incl. Infinity-Cache hits: bases gathered once per window entry",
    }
    # VALU instructions per Fq product (microbenchmark: grid threads, 200
    # products per lane, the largest run) and per mixed add (2^21 GLV points x
    # 8 windows of the 2^20 MSM, one madd per entry)
    if mb and res["valu_insts_per_launch"]:
        g = max(mb)
        per_fqmul = max(mb[g]) / (g / 64 * 200)
        per_madd = res["valu_insts_per_launch"] / (2 * (1 << 20) * 8 / 64)
        res.update({"valu_insts_per_fq_mul": per_fqmul, "valu_insts_per_madd": per_madd,
                    "fq_mul_equiv_per_madd": per_madd / per_fqmul,
                    "fq_mul_equiv_note": "SQ_INSTS_VALU of k_bucket_acc_short per wave-madd / of k_mb_fqmul per "
                                         "wave-product (madds = 2^21 GLV points x 8 windows per MSM)"})
    if dtrace:
        durs = defaultdict(list)
        for f in glob.glob(os.path.join(dtrace, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_bucket_acc_short" in r["Kernel_Name"]:
                    g = int(r["Grid_Size_X"]) if "Grid_Size_X" in r else int(r["Grid_Size"])
                    durs[g].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        if durs:
            res["per_grid_avg_ms"] = {str(g): avg(v) for g, v in durs.items()}
            res["per_grid_launches"] = {str(g): len(v) for g, v in durs.items()}
            res["kernel_ms_per_msm"] = sum(avg(v) for v in durs.values())
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
