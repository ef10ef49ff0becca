"""VALU issue-slot and divergence figures of one kernel from a rocprofv3
--pmc pass of SQ_INSTS_VALU, SQ_INSTS_VALU_INT64, SQ_INSTS_VALU_INT32,
SQ_ACTIVE_INST_VALU, SQ_THREAD_CYCLES_VALU, SQ_WAVE_CYCLES, SQ_WAIT_INST_ANY,
SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE (one pass: 8 SQ + 1 GRBM counters).

* slots: v_mad_u64_u32 (a 64-bit integer VALU instruction, counted by
  SQ_INSTS_VALU_INT64) takes two issue slots of a 32-bit VALU instruction, so
  issue slots = SQ_INSTS_VALU + SQ_INSTS_VALU_INT64;
* valu_busy: SQ_ACTIVE_INST_VALU (quad-cycles, summed over the SIMDs) x 4 /
  (SIMDs x kernel cycles), the kernel cycles from GRBM_GUI_ACTIVE (summed over
  the 8 XCDs: / 8);
* utilization (divergence): SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64),
  rocprofv3's VALUUtilization.
Values are per launch group: the sum over the launches of `per` consecutive
dispatches (the MSM's window-group launches: per = 3) averaged over groups.

    python tools/pmc_valu.py OUT.json DIR KERNEL_SUBSTRING [PER] [MB_KERNEL]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 1024


def main():
    out, d, key = sys.argv[1:4]
    per = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    mbk = sys.argv[5] if len(sys.argv) > 5 else None
    disp = defaultdict(dict)
    mb = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
            if key in r["Kernel_Name"]:
                disp[did][r["Counter_Name"]] = disp[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            elif mbk and mbk in r["Kernel_Name"]:
                mb[did][r["Counter_Name"]] = mb[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(disp)
    groups = [ids[i:i + per] for i in range(0, len(ids) - per + 1, per)]
    if not groups:
        print("no dispatches of", key)
        return 1
    names = sorted({c for v in disp.values() for c in v})
    tot = {c: sum(sum(disp[i].get(c, 0.0) for i in g) for g in groups) / len(groups) for c in names}
    v, v64 = tot.get("SQ_INSTS_VALU", 0.0), tot.get("SQ_INSTS_VALU_INT64", 0.0)
    res = {"kernel_match": key, "launches_per_group": per, "groups": len(groups), "counters_per_group": tot,
           "valu_insts": v, "int64_insts": v64, "issue_slots": v + v64,
           "int64_frac_of_valu": v64 / v if v else None}
    act, thr = tot.get("SQ_ACTIVE_INST_VALU"), tot.get("SQ_THREAD_CYCLES_VALU")
    gui = tot.get("GRBM_GUI_ACTIVE")
    if act and thr:
        res["valu_utilization"] = thr / (act * 64)
    if act and gui:
        res["valu_busy_frac"] = act * 4 / (SIMDS * gui / 8)
    wc, wi = tot.get("SQ_WAVE_CYCLES"), tot.get("SQ_WAIT_INST_ANY")
    if wc and wi:
        res["wait_inst_any_frac_of_wave_cycles"] = wi / wc
    if mb:
        m = max(mb.values(), key=lambda x: x.get("SQ_INSTS_VALU", 0.0))
        res["microbench"] = {"kernel_match": mbk, **m,
                             "int64_frac_of_valu": m.get("SQ_INSTS_VALU_INT64", 0.0) / max(m.get("SQ_INSTS_VALU", 1.0), 1.0)}
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
