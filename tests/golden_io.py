"""Decode tests/golden/*.json (hex strings) into Python ints / limb arrays."""
import json
import os

import numpy as np

from testudo_amd.encoding import fr_array, g1_array, g2_array

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def i(x):
    return int(x, 16)


def g1(p):
    return None if p is None else (i(p[0]), i(p[1]))


def g2(p):
    return None if p is None else ((i(p[0][0]), i(p[0][1])), (i(p[1][0]), i(p[1][1])))


def gt(t):
    return [i(c) for c in t]


def gt_array(t):
    out = np.zeros((12, 6), dtype=np.uint64)
    for k, c in enumerate(t):
        v = i(c)
        out[k] = [(v >> (64 * q)) & (2**64 - 1) for q in range(6)]
    return out.reshape(72)


def fr_arr(xs):
    return fr_array([i(x) for x in xs])


def g1_arr(ps):
    return g1_array([g1(p) for p in ps])


def g2_arr(ps):
    return g2_array([g2(p) for p in ps])


def srs_flat(d):
    """Golden SRS -> the flat canonical layout of include/tpst.h."""
    s = d["srs"]
    parts = [g1_arr([s["g"]]).reshape(-1), g2_arr([s["h"]]).reshape(-1)]
    for lg, lh in zip(s["powers_of_g"], s["powers_of_h"]):
        parts.append(g1_arr(lg).reshape(-1))
        parts.append(g2_arr(lh).reshape(-1))
    parts.append(g1_arr(s["g_mask"]).reshape(-1))
    parts.append(g2_arr(s["h_mask"]).reshape(-1))
    return np.concatenate(parts).astype(np.uint64)
