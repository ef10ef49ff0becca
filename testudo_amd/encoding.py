"""Host-side encoding between Python integers / tuples and the C-ABI limb
layout of include/tpst.h (canonical little-endian u64 limbs; infinity = all
zero).  Points are Python tuples ``(x, y)`` (G2: ``((x0, x1), (y0, y1))``)
or ``None`` for infinity, matching arkworks' affine coordinates.
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1


def int_to_limbs(v: int, n: int) -> list:
    return [(v >> (64 * i)) & M64 for i in range(n)]


def limbs_to_int(a) -> int:
    v = 0
    for i, x in enumerate(a):
        v |= int(x) << (64 * i)
    return v


def fr_array(vals) -> np.ndarray:
    out = np.zeros((len(vals), 4), dtype=np.uint64)
    for i, v in enumerate(vals):
        out[i] = int_to_limbs(int(v), 4)
    return out


def g1_array(points) -> np.ndarray:
    out = np.zeros((len(points), 12), dtype=np.uint64)
    for i, p in enumerate(points):
        if p is not None:
            out[i, :6] = int_to_limbs(p[0], 6)
            out[i, 6:] = int_to_limbs(p[1], 6)
    return out


def g2_array(points) -> np.ndarray:
    out = np.zeros((len(points), 24), dtype=np.uint64)
    for i, p in enumerate(points):
        if p is not None:
            (x0, x1), (y0, y1) = p
            for k, v in enumerate((x0, x1, y0, y1)):
                out[i, 6 * k:6 * k + 6] = int_to_limbs(v, 6)
    return out


def g1_from_array(a):
    a = np.asarray(a, dtype=np.uint64).reshape(-1, 12)
    out = []
    for row in a:
        if not row.any():
            out.append(None)
        else:
            out.append((limbs_to_int(row[:6]), limbs_to_int(row[6:])))
    return out


def g2_from_array(a):
    a = np.asarray(a, dtype=np.uint64).reshape(-1, 24)
    out = []
    for row in a:
        if not row.any():
            out.append(None)
        else:
            v = [limbs_to_int(row[6 * k:6 * k + 6]) for k in range(4)]
            out.append(((v[0], v[1]), (v[2], v[3])))
    return out


def gt_from_array(a) -> list:
    """576-byte GT element -> 12 Fq ints in arkworks tower order."""
    a = np.asarray(a, dtype=np.uint64).reshape(12, 6)
    return [limbs_to_int(r) for r in a]


def gt_array(tower) -> np.ndarray:
    out = np.zeros((12, 6), dtype=np.uint64)
    for i, v in enumerate(tower):
        out[i] = int_to_limbs(v, 6)
    return out.reshape(72)


def ptr(a: np.ndarray):
    import ctypes as C
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(C.c_uint64))
