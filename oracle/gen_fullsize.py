"""Generate the BASELINE-size sqrt-PST fixtures (tests/golden/fullsize_n*.json).

TEST INFRASTRUCTURE ONLY.  Runs the C++ CPU oracle (oracle/cpu, the
arkworks-shaped restatement pinned against oracle/py and the golden vectors)
over the bench's exact inputs, in the shape of /root/reference/benches/pst.rs:48-62:

    Z     = 2^n uniform Fr, SplitMix64 stream seed 0x7E57D0 (tpst_fr_stream)
    point = the next n elements of the same stream
    SRS   = MultilinearPC::setup(ceil(n/2)) from the seeded trapdoor 0x7E57D1
    comm_list, T = Polynomial::commit          (sqrt_pst.rs:117-149)
    v            = Polynomial::eval(point)     (sqrt_pst.rs:105-115)
    U, pst_proof, MippProof = Polynomial::open (sqrt_pst.rs:168-230)

and records the outputs as raw little-endian canonical limb bytes (hex):
the full comm_list only as a SHA-256 digest plus a few sampled rows (it is
2^m_col G1 points), every other output in full.  The oracle's own verifier
must accept the proof before anything is written.

    python3 oracle/gen_fullsize.py 20 24        (n = 24 takes a few minutes)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "cpu"))
import orc  # noqa: E402

OUT = os.path.join(HERE, "..", "tests", "golden")
SEED_Z = 0x7E57D0
SEED_SRS = 0x7E57D1


def hx(a):
    return np.ascontiguousarray(a, dtype=np.uint64).tobytes().hex()


def gen(n):
    nv = (n + 1) // 2
    C = 1 << (n // 2)
    t0 = time.time()
    srs = orc.SRS(nv, SEED_SRS)
    Z, k = orc.fr_stream(SEED_Z, 1 << n)
    pt, _ = orc.fr_stream(SEED_Z, n, k)
    v = orc.pst_eval(Z, n, pt)
    comms, T = orc.pst_commit(srs, Z, n)
    t1 = time.time()
    pr = orc.pst_open(srs, Z, n, pt, comms)
    t2 = time.time()
    assert orc.pst_verify(srs, n, pt, v, pr, T), "oracle rejects its own proof"
    rows = sorted({0, 1, C // 2 + 1, C - 1})
    d = {
        "n": n, "srs_nv": nv, "seed_z": SEED_Z, "seed_srs": SEED_SRS,
        "generator": "oracle/gen_fullsize.py (C++ CPU oracle, %d threads)" % orc.load().orc_threads(),
        "oracle_seconds": {"commit": round(t1 - t0, 2), "open": round(t2 - t1, 2)},
        "point": hx(pt), "eval": hx(v),
        "comms_sha256": hashlib.sha256(np.ascontiguousarray(comms).tobytes()).hexdigest(),
        "comms_rows": rows, "comms_sampled": [hx(comms[r]) for r in rows],
        "T": hx(T), "U": hx(pr["U"]), "pst_proof": hx(pr["pst_proof"]),
        "comms_t": hx(pr["comms_t"]), "comms_u": hx(pr["comms_u"]),
        "final_a": hx(pr["final_a"]), "final_h": hx(pr["final_h"]), "pst_proof_h": hx(pr["pst_proof_h"]),
    }
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, "fullsize_n%d.json" % n)
    with open(path, "w") as f:
        json.dump(d, f, indent=0)
    print("wrote", path, "commit %.1fs open %.1fs" % (t1 - t0, t2 - t1), flush=True)


if __name__ == "__main__":
    for a in sys.argv[1:] or ["20"]:
        gen(int(a))
