"""CPU tests of the drop-in boundary: libtpst.so loads, exports every symbol
include/tpst.h declares, and the Python binding mirrors it.  No compute calls
(there is no GPU here); host-only entry points (transcript, input stream)
are exercised against the oracle."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tpst.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tpst_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for must in ("tpst_create", "tpst_g1_msm", "tpst_multi_pairing", "tpst_poly_commit", "tpst_poly_open",
                 "tpst_pst_verify", "tpst_srs_setup"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    from testudo_amd import _lib
    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    from testudo_amd import _lib
    assert sorted(_lib.exported_symbols()) == declared_symbols()


def test_no_device_is_reported_cleanly():
    from testudo_amd import _lib
    lib = _lib.load()
    if lib.tpst_device_count() > 0:
        pytest.skip("a GPU is present")
    h = C.c_void_p()
    assert lib.tpst_create(0, C.byref(h)) == -2  # TPST_E_NODEV, no abort


def test_host_transcript_matches_oracle():
    import bls377 as O
    import golden_io as G
    from testudo_amd.encoding import g1_array
    from testudo_amd.sqrt_pst import PoseidonTranscript
    d = G.load("transcript.json")
    tr = PoseidonTranscript()
    tr.append_g1(g1_array([G.g1(d["append_g1"])])[0])
    c1 = tr.challenge_scalar()
    assert sum(int(x) << (64 * k) for k, x in enumerate(c1)) == G.i(d["c1"])
    tr.append_gt(G.gt_array(d["append_gt"]))
    assert sum(int(x) << (64 * k) for k, x in enumerate(tr.challenge_scalar())) == G.i(d["c2"])
    assert sum(int(x) << (64 * k) for k, x in enumerate(tr.challenge_scalar())) == G.i(d["c3"])
    del O


def test_product_stream_matches_oracle():
    import orc
    from testudo_amd.sqrt_pst import fr_stream
    a, k1 = fr_stream(0x7E57D0, 50)
    b, k2 = orc.fr_stream(0x7E57D0, 50)
    assert np.array_equal(a, b) and k1 == k2


def test_one_hip_runtime_per_process():
    """Loading libtpst pulls torch's HIP runtime in first (testudo_amd/_lib.py),
    so the library and torch share one libamdhip64 / libhsa-runtime64: two
    runtimes in one process leave torch without a GPU and make device
    pointers and streams unshareable."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from testudo_amd import _lib; _lib.load()\n"
            "maps = open('/proc/self/maps').read().splitlines()\n"
            "libs = sorted(set(l.split()[-1] for l in maps if 'libamdhip64' in l))\n"
            "print(len(libs), libs)\n") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("1 "), r.stdout
