"""The RNS chain engine's tables (testudo_amd/csrc/rns_ops.inc) are what
tools/gen_rns_ops.py renders after checking every op through an exact model
of rns_engine.h's arithmetic (every 64-bit accumulator, every value bound,
both base extensions, the conversions in and out); here the committed file
must equal the rendering, and a chain of model stages (outputs feeding the
next stage's inputs, as in k_chain_final_rns) must stay exact and bounded."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_rns_ops as G  # noqa: E402


def test_rns_tables_match_checked_rendering():
    text, stats = G.render()
    with open(G.INC_PATH) as f:
        assert f.read() == text, "rns_ops.inc is stale: run python tools/gen_rns_ops.py"
    assert any("CYC_SQR" in s for s in stats)


def test_rns_model_chain_stays_exact_and_bounded():
    random.seed(7)
    built, rp, progs, kin, kout_slot, _, _ = G.check_all()
    kres = [G.residues(k * G.MB % G.P) for k in rp.consts]
    W = G.W
    a = W.rnd(12)
    b = W.rnd(12)
    ra = [G.residues(G.to_m(v)) for v in a]
    rb = [G.residues(G.to_m(v)) for v in b]
    ref = W.t2p(a)
    fb = W.t2p(b)
    for step in range(6):
        name = "F12_MUL" if step % 2 else "F12_SQR"
        env = {"A": ra, "B": rb, "K": kres}
        out = G.run_op(rp, progs[name], env, None)
        ra = [out[k] for k in range(12)]
        ref = G.O.f12_mul(ref, fb if name == "F12_MUL" else ref)
        for k in range(12):
            x = G.crt(ra[k])
            assert x < G.N1
            assert x % G.P == W.p2t(ref)[k] * G.MB % G.P
    # and out through the store path: canonical field.h Montgomery limbs
    kout = kres[kout_slot]
    for k in range(12):
        t = [G.red64(ra[k][ch] * kout[ch], ch) for ch in range(G.LANES)]
        assert G.store_model(G.mont(t)) == W.p2t(ref)[k] * G.RQ % G.P
