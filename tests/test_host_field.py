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


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_host_mont_adx_matches_cxx(tmp_path):
    """The transcript's MULX / ADCX / ADOX Montgomery product
    (csrc/host_mont_adx.inc, tools/gen_mont_adx.py) equals the __int128 CIOS
    product on 300 000 random inputs below 2p, 0, and 2p - 1 / p - 1 (the
    lazy range the Poseidon permutation feeds it); skipped on a CPU without
    BMI2 / ADX, where the library uses the C++ product."""
    exe = str(tmp_path / "test_mont_adx")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-attributes", "-I" + os.path.join(ROOT, "testudo_amd", "csrc"),
                    "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp", "test_mont_adx.cpp"),
                    "-o", exe], check=True)
    r = subprocess.run([exe, "300000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "skip" in r.stdout or "mismatches 0 of 300000" in r.stdout, r.stdout
