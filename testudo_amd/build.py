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
# A/B builds (experiments): TPST_BUILD_TAG=x builds build_x/ -> libtpst_x.so
# with TPST_EXTRA_FLAGS added (e.g. "-DTPST_F29_2ACC=0"); load it with
# TPST_LIB_PATH.  The product build is the untagged one.
_TAG = os.environ.get("TPST_BUILD_TAG", "")
BUILD = os.path.join(HERE, "build_" + _TAG if _TAG else "build")
LIB = os.path.join(HERE, "libtpst_%s.so" % _TAG if _TAG else "libtpst.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("TPST_ARCH", "gfx950")


def _host_isa_flags() -> list:
    """x86-64-v3 + ADX for the host code (the Poseidon transcript's 768-bit
    products between MIPP rounds) only when TPST_HOST_ISA=v3 asks for it: the
    library then needs AVX2 / BMI2 / ADX on every machine that loads it.  The
    default is the baseline ISA, which runs anywhere (the __int128 code is
    correct without those extensions)."""
    if os.environ.get("TPST_HOST_ISA", "") == "v3":
        return ["-Xarch_host", "-march=x86-64-v3", "-Xarch_host", "-madx"]
    return []


FLAGS = (["-std=c++17", "-O3", "--offload-arch=" + ARCH, "-fPIC", "-Wno-unused-result"] + _host_isa_flags() +
         ["-I" + CSRC, "-I" + os.path.join(ROOT, "include")] + os.environ.get("TPST_EXTRA_FLAGS", "").split())


def _includes(path: str, seen: set) -> None:
    """Transitive local #includes of a source or header (csrc/ and include/)."""
    for inc in re.findall(r'#include "([^"]+)"', open(path).read()):
        for d in (os.path.dirname(path), CSRC, os.path.join(ROOT, "include")):
            f = os.path.join(d, inc)
            if os.path.exists(f):
                f = os.path.abspath(f)
                if f not in seen:
                    seen.add(f)
                    _includes(f, seen)
                break


def _src_mtime(src: str) -> float:
    """newest mtime over a .hip file and everything it includes."""
    seen = {os.path.abspath(src)}
    _includes(src, seen)
    return max(os.path.getmtime(f) for f in seen)


def _compile(src: str) -> str:
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= _src_mtime(src):
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
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", LIB + ".tmp"] + objs + [
            "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]
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
