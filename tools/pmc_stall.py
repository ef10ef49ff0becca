"""Summarise a rocprofv3 --pmc pass of the SQ stall counters per kernel.

    python tools/pmc_stall.py OUT.json DIR_PMC [kernel-substring ...]

Counters (one pass, 8 SQ slots): SQ_WAVE_CYCLES, SQ_WAIT_ANY (wave parked on
s_waitcnt / barrier: memory latency), SQ_WAIT_INST_ANY (issue stall: operand
dependency or pipe busy), SQ_ACTIVE_INST_ANY / _VALU (cycles issuing),
SQ_INSTS_VMEM_RD, SQ_INSTS_SALU, SQ_BUSY_CYCLES.  WAIT_ANY + WAIT_INST_ANY +
ACTIVE_INST_ANY ~= WAVE_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots),
so the three fractions attribute every wave cycle.
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    out, d = sys.argv[1], sys.argv[2]
    keys = sys.argv[3:] or ["k_bucket_acc_short", "k_bucket_acc_chunk"]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            k = next((k for k in keys if k in name), None)
            if k is None:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r.get("Dispatch_Id", ""))
    res = {}
    for k, v in agg.items():
        wc = v.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        res[k] = {
            "dispatches": len(disp[k]),
            "counters": v,
            "frac_issuing": v.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
            "frac_issue_stall": v.get("SQ_WAIT_INST_ANY", 0.0) / wc,
            "frac_waitcnt": v.get("SQ_WAIT_ANY", 0.0) / wc,
            "valu_share_of_issue": v.get("SQ_ACTIVE_INST_VALU", 0.0) / (v.get("SQ_ACTIVE_INST_ANY", 0.0) or 1.0),
        }
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
