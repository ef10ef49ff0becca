"""Microbenchmark probe: Fq multiply variants (latency / throughput / check)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from testudo_amd import Context
ctx = Context(0)
# check kind 3: all ones
ms = ctx.microbench(3, 256 * 64, 1)
import ctypes as C
print("check kernel ran", ms)
for kind, name in ((0, "fips"), (2, "fips_ilp2"), (1, "madd")):
    it = 2000
    lat = ctx.microbench(kind, 64, it) * 1e3 / it
    out = []
    for wpc in (4, 8, 16):
        thr = 256 * wpc * 64
        ms = ctx.microbench(kind, thr, 200)
        out.append("%d w/CU %.2f G/s" % (wpc, thr * 200 / ms / 1e6))
    print("%-10s latency %.3f us | %s" % (name, lat, " | ".join(out)), flush=True)
