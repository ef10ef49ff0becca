"""pytest setup: the `gpu` marker and import paths.

`-m "not gpu"` runs the oracle-vs-golden checks, host logic and the C-ABI
load/export checks (no GPU needed); `-m gpu` runs the parity tests that call
libtpst on an MI355X.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle", "py"), os.path.join(ROOT, "oracle", "cpu")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libtpst.so")


@pytest.fixture(scope="session")
def ctx():
    from testudo_amd import Context
    c = Context(0)
    yield c
    c.close()
