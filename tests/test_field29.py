"""field29.h (the radix-2^29 Fq of the MSM accumulation, the MSM tail and
the wave engine's products) checked on the host against Python integers:
Montgomery product / square / add / sub, the one-reduction sum of two
products (mul_sum / mul_sub), the conversions from and to
field.h's layout (R = 2^384 <-> 2^377), the packed bucket format (pack377 /
unpack377: the R = 2^377 value's bits in 12 words), the binary-GCD inverse, and the wave
engine's stage product on unreduced operands (a form of weight w is < w p;
the engine feeds products with w_x w_y <= 64, squares with w <= 8)."""
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0x01AE3A4617C510EAC63B05C06CA1493B1A22D9F300F5138F1EF3622FBA094800170B5D44300000008508C00000000001
R = 1 << 384
RI = pow(R, -1, P)


def _w(v):
    return " ".join("%x" % ((v >> (32 * i)) & 0xFFFFFFFF) for i in range(12))


def _parse(line):
    return sum(int(t, 16) << (32 * i) for i, t in enumerate(line.split()))


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("f29") / "test_field29")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "testudo_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "test_field29.cpp"), "-o", out], check=True)
    return out


def _run(exe, rows):
    inp = "%d\n" % len(rows) + "\n".join("%d %s %s" % (w, _w(a), _w(b)) for w, a, b in rows)
    return subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.split("\n")


def test_field29_ops_and_inverse(exe):
    rng = random.Random(29)
    vals = [(0, 0), (1, P - 1), (P - 1, P - 1), (P - 1, 1), (1 << 376, 3)]
    vals += [(rng.randrange(P), rng.randrange(P)) for _ in range(2000)]
    out = _run(exe, [(0, a * R % P, b * R % P) for a, b in vals])
    for k, (a, b) in enumerate(vals):
        got = [_parse(out[12 * k + j]) for j in range(12)]
        exp = [a * b % P * R % P, a * a % P * R % P, (a + b) % P * R % P, (a - b) % P * R % P, a * R % P,
               (pow(a, -1, P) * R % P) if a else 0, (a * b + a * a) % P * R % P, (a * b - b * b) % P * R % P,
               a * (1 << 377) % P, a * R % P, (-a) % P * R % P, a * R % P]
        assert got == exp, (a, b)


def test_field29_wave_stage_products_on_wide_operands(exe):
    rng = random.Random(30)
    rows = []
    for wx in (1, 2, 4, 8, 16, 32, 64):
        wy = max(1, 64 // wx)
        rows += [(1, rng.randrange(wx * P), rng.randrange(wy * P)) for _ in range(300)]
        rows.append((1, wx * P - 1, wy * P - 1))
    out = _run(exe, rows)
    for k, (_, a, b) in enumerate(rows):
        assert _parse(out[2 * k]) == a * b * RI % P
        if a < 8 * P:
            assert _parse(out[2 * k + 1]) == a * a * RI % P
