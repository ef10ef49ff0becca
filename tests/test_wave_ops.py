"""The wave-engine stage tables (testudo_amd/csrc/wave_ops.inc) are what
tools/gen_wave_ops.py derives from the tower formulas: every op -- Fq12
multiply, the all-squares Fq12 / cyclotomic squarings, Frobenius maps, the
inversion chain and the G2Prepared doubling / addition steps -- is checked
numerically against the pure-Python oracle (oracle/py/bls377.py) while the
tables are rendered, and the committed file must equal the rendering."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_wave_ops  # noqa: E402


def test_wave_ops_tables_match_checked_rendering():
    text, stats = gen_wave_ops.render()
    with open(gen_wave_ops.INC_PATH) as f:
        assert f.read() == text, "wave_ops.inc is stale: run python tools/gen_wave_ops.py"
    sq = [s for s in stats if "squares " in s]
    assert any("CYC_SQR" in s for s in sq) and any("F12_SQR" in s for s in sq)
