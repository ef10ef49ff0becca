"""Build libtpst.so (HIP, gfx950) in-tree: testudo_amd/libtpst.so.

Each .hip translation unit is compiled with hipcc --offload-arch=gfx950 in
parallel and re-used while it is newer than every header it could include;
the objects are linked into one shared library that exports the C-ABI of
include/tpst.h.  Cross-compiles without a GPU.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libtpst.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("TPST_ARCH", "gfx950")
FLAGS = ["-std=c++17", "-O3", "--offload-arch=" + ARCH, "-fPIC", "-Wno-unused-result",
         "-I" + CSRC, "-I" + os.path.join(ROOT, "include")]


def _deps_mtime() -> float:
    files = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.inc"))
    files.append(os.path.join(ROOT, "include", "tpst.h"))
    return max(os.path.getmtime(f) for f in files)


def _src_mtime(src: str) -> float:
    """mtime of a .hip file and of any .hip it #includes (msm_g2.hip)."""
    t = os.path.getmtime(src)
    for inc in re.findall(r'#include "([^"]+\.hip)"', open(src).read()):
        t = max(t, os.path.getmtime(os.path.join(os.path.dirname(src), inc)))
    return t


def _compile(src: str, hdr_mtime: float) -> str:
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(_src_mtime(src), hdr_mtime):
        return obj
    cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s" % (src, r.stderr[-6000:]))
    os.replace(obj + ".tmp", obj)
    return obj


def build(verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hdr = _deps_mtime()
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", LIB + ".tmp"] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stderr[-4000:])
        os.replace(LIB + ".tmp", LIB)
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    try:
        build()
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
