"""Generate tests/golden/*.json from the pure-Python oracle.

TEST INFRASTRUCTURE ONLY.  Every value is produced by oracle/py (first-
principles restatement; see bls377.py / pst.py headers).  The reference's own
known-answer test (dense_mlpoly.rs:609-623: Z=[1,2,1,4], r=[4,3] -> 28) is
included verbatim as data.  Run:  python3 oracle/py/gen_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import bls377 as O  # noqa: E402
import pst as P  # noqa: E402

OUT = os.path.join(HERE, "..", "..", "tests", "golden")


def h(v):
    return "%x" % v


def g1h(p):
    return None if p is None else [h(p[0]), h(p[1])]


def g2h(p):
    return None if p is None else [[h(p[0][0]), h(p[0][1])], [h(p[1][0]), h(p[1][1])]]


def gth(f):
    return [h(c) for c in O.fq12_to_tower(f)]


def dump(name, obj):
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, name), "w") as f:
        json.dump(obj, f, indent=0)
    print("wrote", name)


def main():
    # reference KAT, dense_mlpoly.rs:609-623
    dump("kat_dense_eval.json", {"source": "reference src/dense_mlpoly.rs:609-623", "Z": [1, 2, 1, 4],
                                 "r": [4, 3], "eval": 28})

    # MSMs
    s, _ = P.fr_stream(101, 33)
    b, _ = P.fr_stream(102, 33)
    bases = [O.g1_mul(O.G1_GEN, x) for x in b]
    bases[5] = None  # an infinity base
    s[7] = 0          # a zero scalar
    msm = O.g1_msm(bases, s)
    s2, _ = P.fr_stream(103, 9)
    b2, _ = P.fr_stream(104, 9)
    bases2 = [O.g2_mul(O.G2_GEN, x) for x in b2]
    msm2 = O.g2_msm(bases2, s2)
    dump("msm.json", {"g1": {"bases": [g1h(p) for p in bases], "scalars": [h(x) for x in s], "out": g1h(msm)},
                      "g2": {"bases": [g2h(p) for p in bases2], "scalars": [h(x) for x in s2], "out": g2h(msm2)}})

    # pairings (ark chain checked against direct exponentiation by 3(p^12-1)/r)
    ps = [O.g1_mul(O.G1_GEN, 1 + i) for i in range(3)]
    qs = [O.g2_mul(O.G2_GEN, 7 + i) for i in range(3)]
    e = O.multi_pairing(ps, qs)
    assert e == O.f12_mul(O.f12_mul(O.pairing_textbook(ps[0], qs[0]), O.pairing_textbook(ps[1], qs[1])),
                          O.pairing_textbook(ps[2], qs[2]))
    dump("pairing.json", {"g1": [g1h(p) for p in ps], "g2": [g2h(q) for q in qs], "gt": gth(e),
                          "e_gen": gth(O.pairing(O.G1_GEN, O.G2_GEN))})

    # Poseidon transcript
    tr = P.PoseidonTranscript()
    tr.append_g1(O.G1_GEN)
    c1 = tr.challenge_scalar()
    tr.append_gt(e)
    c2 = tr.challenge_scalar()
    c3 = tr.challenge_scalar()
    dump("transcript.json", {"append_g1": g1h(O.G1_GEN), "c1": h(c1), "append_gt": gth(e), "c2": h(c2), "c3": h(c3)})

    # full sqrt-PST commit/open (benches/pst.rs flow) for n = 4..7
    for n in (4, 5, 6, 7):
        Z, k = P.fr_stream(P.SEED, 1 << n)
        r, _ = P.fr_stream(P.SEED, n, k)
        srs = P.SRS((n + 1) // 2)
        pl = P.Polynomial(Z)
        v = pl.eval(r)
        comms, T = pl.commit(srs)
        tr = P.PoseidonTranscript()
        U, pst_proof, mipp = pl.open(tr, comms, srs, r, T)
        assert P.Polynomial.verify(P.PoseidonTranscript(), srs, U, r, v, pst_proof, mipp, T)
        dump("sqrt_pst_n%d.json" % n, {
            "n": n, "Z_seed": P.SEED, "srs_seed": P.SEED + 1, "srs_nv": (n + 1) // 2,
            "Z": [h(x) for x in Z], "point": [h(x) for x in r], "eval": h(v),
            "comms": [g1h(c) for c in comms], "T": gth(T), "U": g1h(U),
            "pst_proof": [g2h(x) for x in pst_proof],
            "comms_t": [[gth(a), gth(b_)] for a, b_ in mipp["comms_t"]],
            "comms_u": [[g1h(a), g1h(b_)] for a, b_ in mipp["comms_u"]],
            "final_a": g1h(mipp["final_a"]), "final_h": g2h(mipp["final_h"]),
            "pst_proof_h": [g1h(x) for x in mipp["pst_proof_h"]],
            "srs": {"g": g1h(srs.g), "h": g2h(srs.h), "g_mask": [g1h(x) for x in srs.g_mask],
                    "h_mask": [g2h(x) for x in srs.h_mask],
                    "powers_of_g": [[g1h(x) for x in lvl] for lvl in srs.powers_of_g],
                    "powers_of_h": [[g2h(x) for x in lvl] for lvl in srs.powers_of_h]},
        })


if __name__ == "__main__":
    main()
