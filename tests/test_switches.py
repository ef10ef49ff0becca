"""The three environment switches libtpst still reads (INTEGRATION.md
"Tunables"), each run at its non-default value in a child process (they are
read once per process) and checked bit-exact against the default path's
fixtures / the CPU oracle:

* TPST_OPEN_TRACE=1 -- diagnostics only: the per-round trace is printed and
  the n = 20 proof is unchanged (fixture fullsize_n20.json);
* TPST_COMMIT_TABLE=0 at n = 20 and n = 24 (the opening builds the fold
  table itself instead of the commit) -- same proofs as the fixtures;
* TPST_ACC_LDS=0 -- the register-prefetch MSM accumulation instead of the
  default LDS staging, 2^17 + 37 points vs the oracle.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

_OPEN = r'''
import hashlib, json, sys
import numpy as np
sys.path.insert(0, %(root)r); sys.path.insert(0, %(root)r + "/tests")
import golden_io as G
from testudo_amd import Context
from testudo_amd import sqrt_pst as S
n = %(n)d
d = G.load("fullsize_n%%d.json" %% n)
ctx = Context(0)
S.srs_setup(ctx, d["srs_nv"], d["seed_srs"])
Z, k = S.fr_stream(d["seed_z"], 1 << n)
pt, _ = S.fr_stream(d["seed_z"], n, k)
pl = S.Polynomial.from_evaluations(ctx, Z)
del Z
comms, T = pl.commit()
pl.eval(pt)
U, pst, mipp = pl.open(S.PoseidonTranscript(), comms, pt, T)
h = lambda a: np.ascontiguousarray(a, dtype=np.uint64).tobytes().hex()
ok = {"comms": hashlib.sha256(comms.tobytes()).hexdigest() == d["comms_sha256"], "T": h(T) == d["T"],
      "U": h(U) == d["U"], "pst": h(pst) == d["pst_proof"], "comms_t": h(mipp.comms_t) == d["comms_t"],
      "comms_u": h(mipp.comms_u) == d["comms_u"], "final_a": h(mipp.final_a) == d["final_a"],
      "final_h": h(mipp.final_h) == d["final_h"], "pst_proof_h": h(mipp.pst_proof_h) == d["pst_proof_h"]}
print("RESULT " + json.dumps(ok))
'''

_MSM = r'''
import json, sys
import numpy as np
sys.path.insert(0, %(root)r); sys.path.insert(0, %(root)r + "/oracle/cpu")
import orc
from testudo_amd import Context
ctx = Context(0)
n = (1 << 17) + 37
k, _ = orc.fr_stream(91, n)
s, _ = orc.fr_stream(92, n)
bases = ctx.g1_mul_generator(k)
ok = {"msm": bool(np.array_equal(ctx.g1_msm(bases, s), orc.g1_msm(bases, s, parallel=True)))}
s[::3] = 0
s[1::3, 1:] = 0
ok["skewed"] = bool(np.array_equal(ctx.g1_msm(bases, s), orc.g1_msm(bases, s, parallel=True)))
print("RESULT " + json.dumps(ok))
'''


def _run(script, env_extra, timeout=240):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, env=env, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    return json.loads(line[7:]), r.stderr


def test_open_trace_leaves_proof_unchanged():
    ok, err = _run(_OPEN % {"root": ROOT, "n": 20}, {"TPST_OPEN_TRACE": "1"})
    assert all(ok.values()), ok
    assert err.count("open round") == 10, err[-2000:]


@pytest.mark.parametrize("n,val", [(20, "0"), (24, "0")])
def test_commit_table_forced_off(n, val):
    ok, _ = _run(_OPEN % {"root": ROOT, "n": n}, {"TPST_COMMIT_TABLE": val})
    assert all(ok.values()), ok


def test_acc_register_prefetch_msm_vs_oracle():
    ok, _ = _run(_MSM % {"root": ROOT}, {"TPST_ACC_LDS": "0"})
    assert all(ok.values()), ok
