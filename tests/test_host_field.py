"""Host build of csrc/field.h (the same header the HIP kernels use) checked
on the CPU: the constant-flow modular inverse over Fq and Fr."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_constant_flow_inverse_host(tmp_path):
    exe = str(tmp_path / "test_inv")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "testudo_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "test_inv.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe, "5000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fq_bad 0 fr_bad 0" in r.stdout
