"""Compile-time register / scratch report for every kernel of libtpst.

Runs hipcc on each csrc/*.hip (device side only, gfx950) with
-Rpass-analysis=kernel-resource-usage and tabulates, per kernel: VGPRs,
AGPRs, SGPRs, VGPR / SGPR spills, private scratch bytes per lane, the
compiler's occupancy (waves per SIMD) and LDS bytes per workgroup.

  python tools/kernel_resources.py [--out profiles/r05/kernel_resources.txt]
                                   [--only msm.hip,...] [--check]

--check exits non-zero when a kernel listed in HOT has VGPR spills or private
scratch (the accumulation / fixup / reduction kernels of the MSMs and the
commit).  SGPR spills are listed apart: they go to VGPR lanes
(v_writelane / v_readlane), no memory.
CPU only: cross-compiles, needs no GPU.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "testudo_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# kernels that must be free of spills and scratch: the bucket
# accumulations of the variable-base MSM (K2) and of the commit (K1), their
# fixups and the bucket reductions
HOT = [
    "k_bucket_acc_short<Fp<FqCfg>, 2, true>",
    "k_bucket_acc_short_lds<2, true>",
    "k_bucket_acc_chunk<Fp<FqCfg>, 2, true>",
    "k_bucket_acc_chunk_lds<2>",
    "k_bucket_fixup_short<Fp<FqCfg> >",
    "k_bucket_fixup_quad<Fp<FqCfg> >",
    "k_bucket_fixup_long<Fp<FqCfg> >",
    "k_bucket_fixup<Fp<FqCfg> >",
    "k_seg_reduce_lane<Fp<FqCfg> >",
    "k_seg_reduce_quad<Fp<FqCfg> >",
    "k_seg_run_lane<Fp<FqCfg> >",
    "k_seg_run_quad<Fp<FqCfg> >",
    "k_group_reduce_quad<Fp<FqCfg>, 256>",
    "k_lift_add_quad<Fp<FqCfg> >",
]

FIELDS = {
    "VGPRs": "vgpr", "AGPRs": "agpr", "TotalSGPRs": "sgpr", "ScratchSize [bytes/lane]": "scratch",
    "Occupancy [waves/SIMD]": "occ", "SGPRs Spill": "sspill", "VGPRs Spill": "vspill",
    "LDS Size [bytes/block]": "lds",
}


def _demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.strip().split("\n") if r.returncode == 0 else list(names)


def report(src: str) -> list:
    flags = ["-std=c++17", "-O3", "--offload-arch=gfx950", "--cuda-device-only", "-c", "-o", os.devnull,
             "-I" + CSRC, "-I" + os.path.join(ROOT, "include"), "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run([HIPCC] + flags + [src], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s" % (src, r.stderr[-3000:]))
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"mangled": m.group(1), "file": os.path.basename(src)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+(.+?): (\S+) \[-Rpass-analysis", line)
        if m and cur is not None and m.group(1).strip() in FIELDS:
            v = m.group(2)
            cur[FIELDS[m.group(1).strip()]] = int(v) if v.lstrip("-").isdigit() else v
    for row, d in zip(rows, _demangle([x["mangled"] for x in rows])):
        d = d[5:] if d.startswith("void ") else d
        row["name"] = d.replace("tpst::", "").replace("(anonymous namespace)::", "")
    return rows


def short(name: str) -> str:
    """kernel name with template arguments, without the parameter list"""
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i]
    return name


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="comma-separated .hip basenames")
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    if a.only:
        keep = set(a.only.split(","))
        srcs = [s for s in srcs if os.path.basename(s) in keep]
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        rows = [r for rs in ex.map(report, srcs) for r in rs]
    hdr = "%-14s %-72s %5s %4s %5s %6s %6s %7s %4s %7s" % (
        "file", "kernel", "vgpr", "agpr", "sgpr", "vspill", "sspill", "scratch", "occ", "lds")
    lines = [hdr, "-" * len(hdr)]
    bad, lanes = [], []
    for r in rows:
        k = short(r["name"])
        lines.append("%-14s %-72s %5s %4s %5s %6s %6s %7s %4s %7s" % (
            r["file"], k[:72], r.get("vgpr"), r.get("agpr"), r.get("sgpr"), r.get("vspill"), r.get("sspill"),
            r.get("scratch"), r.get("occ"), r.get("lds")))
        if k in HOT and (r.get("vspill") or r.get("scratch")):
            bad.append(k)
        elif k in HOT and r.get("sspill"):
            lanes.append("%s (%s)" % (k, r.get("sspill")))
    text = "\n".join(lines) + "\n"
    seen = {short(r["name"]) for r in rows}
    missing = [h for h in HOT if h not in seen] if not a.only or "msm.hip" in a.only else []
    if missing:
        text += "\nHOT kernels not found (renamed?):\n" + "\n".join("  " + m for m in missing) + "\n"
        bad += missing
    if lanes:
        text += ("\nHOT kernels with SGPR spills (to VGPR lanes: v_writelane / v_readlane, no scratch memory):\n" +
                 "\n".join("  " + b for b in lanes) + "\n")
    if bad:
        text += "\nHOT kernels with spills or scratch:\n" + "\n".join("  " + b for b in bad) + "\n"
    else:
        text += "\nHOT kernels: no spills, no scratch (%d checked)\n" % len(HOT)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(text)
    sys.stdout.write(text)
    return 1 if (a.check and bad) else 0


if __name__ == "__main__":
    sys.exit(main())
