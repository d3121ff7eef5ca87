"""Host arithmetic of the round hand-off (repo csrc/hfield.hpp), checked on the
CPU against Python big integers: hlimbs_to_fe (limb sums at 32-bit positions ->
Montgomery image; its 512-bit REDC fast path and the general path) and the
unreduced product sums of the host rounds (mac_wide + wide_to_fe). The checker
is compiled from tests/native/host_arith_check.cpp with the ROCm clang (host
code only, no GPU)."""
from __future__ import annotations

import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "host_arith_check.cpp")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
MODULI = [
    0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001,  # BN254 Fr
    0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47,  # BN254 Fq
    0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,  # BLS12-381 Fr
]
R = 1 << 256


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if not os.path.exists(CLANG):
        pytest.skip("ROCm clang++ not present")
    exe = str(tmp_path_factory.mktemp("hac") / "host_arith_check")
    subprocess.run([CLANG, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "zk-research-implementations_amd", "csrc"), SRC,
                    "-o", exe], check=True)
    return exe


def _run(exe: str, field: int, lines: list[str]) -> list[int]:
    out = subprocess.run([exe, str(field)], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
    vals = []
    for ln in out.stdout.split("\n"):
        if ln.strip():
            l0, l1, l2, l3 = (int(x, 16) for x in ln.split())
            vals.append(l0 | l1 << 64 | l2 << 128 | l3 << 192)
    return vals


@pytest.mark.parametrize("field", [0, 1, 2])
def test_limb_sums_to_field(checker, field):
    p = MODULI[field]
    rng = random.Random(7 + field)
    lines, want = [], []
    # the shapes the library hands over: unreduced product sums (9 limb sums of a
    # matrix-core step, 17 words of a VALU step, 18 from the host rounds' 9 x 64-bit
    # accumulators) and element sums (8 limb sums)
    cases = [(9, 45, 1), (9, 64, 1), (17, 40, 1), (17, 64, 1), (18, 32, 1), (8, 50, 0), (8, 64, 0)]
    for L, bits, product in cases:
        for _ in range(60):
            w = [rng.getrandbits(bits) for _ in range(L)]
            if rng.random() < 0.2:  # edge values: all ones / zeros in the top word
                w[-1] = (1 << bits) - 1 if rng.random() < 0.5 else 0
            v = sum(x << (32 * i) for i, x in enumerate(w))
            lines.append(f"{L} {product} " + " ".join(f"{x:x}" for x in w))
            # product sums are of two Montgomery images (v = a b R^2): image of a b is v R^-1;
            # element sums (v = a R): image v
            want.append(v * pow(R, -1, p) % p if product else v % p)
    # either side of the 512-bit REDC fast path's bound (value < p R)
    for v in [p * R - 1, p * R, p * R + 1, p * R - (1 << 255), 2**512 - 1, p * p, 3 * (p - 1) ** 2, 0, 1]:
        w = [(v >> (32 * i)) & 0xFFFFFFFF for i in range(16)]
        lines.append("16 1 " + " ".join(f"{x:x}" for x in w))
        want.append(v * pow(R, -1, p) % p)
    assert _run(checker, field, lines) == want


@pytest.mark.parametrize("field", [0, 1, 2])
def test_unreduced_product_sums(checker, field):
    p = MODULI[field]
    rng = random.Random(11 + field)
    lines, want = [], []
    for _ in range(200):
        xs = [rng.randrange(p) if rng.random() < 0.9 else p - 1 for _ in range(4)]
        lines.append("M " + " ".join(" ".join(f"{(x >> (64 * k)) & (2**64 - 1):x}" for k in range(4)) for x in xs))
        want.append((xs[0] * xs[1] + xs[2] * xs[3]) * pow(R, -1, p) % p)
    assert _run(checker, field, lines) == want
