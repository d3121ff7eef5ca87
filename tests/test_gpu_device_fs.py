"""Device-resident Fiat-Shamir (ZK_DEVICE_FS=1,
zk-research-implementations_amd/csrc/dfs.hpp).

With the knob on, every step of the persistent double-step tail (k_gkr_dtail)
but its last draws the next step's challenges on the device: the block that
counts in last reduces the eight product sums, interpolates both rounds
(univariate_polynomial_dense.rs:48-74, trimmed :14-18), absorbs the canonical
coefficients after the previous digest and runs Keccak-f on the device
(fiat_shamir_transcript.rs:23-37), and relays (r_m, r_m+1, r_m r_m+1, digest,
claim) to the next step without a host round trip (sum_check_protocol.rs:96-108).
The host then replays the logged rounds into its own transcript and fails with
ZK_EDEVICE if any device challenge differs from the one it draws.

Checked here against the C oracle (oracle/zk_oracle.c, the restatement of
gkr_prove, sum_check_protocol.rs:86-166):
* all three fields, odd and even round counts, with the last rounds on the
  host (ZK_HOST_ROUNDS=4, default) and all on the device (0);
* every trimmed coefficient count the device absorbs: 3 (random tables),
  2 (S = 1: each round polynomial is linear), 1 (A, S constant), 0 (zero tables);
* a caller transcript holding earlier bytes of every length around the
  136-byte Keccak rate (the host's absorbs cross rate blocks before the tail;
  the device continues from the digest of the last challenge);
* that the device really drew the challenges (stats: device_fs_rounds).
"""
from __future__ import annotations

import numpy as np
import pytest

import coracle as co

import zk_amd
from zk_amd import ProductPoly, SumPoly, Transcript

pytestmark = pytest.mark.gpu


def _tables(field: int, n: int, shape: str) -> list:
    N = 1 << n
    base = [co.synth(field, 31, t, 0, N) for t in range(4)]
    zero = np.zeros_like(base[0])
    if shape == "random":
        return base
    if shape == "linear":  # A S + 0 with S = 1: every round polynomial has degree 1 (two coefficients)
        return [base[0], co.to_limbs([1] * N), zero, zero]
    if shape == "constant":  # A = 5, S = 7: constant round polynomials (one coefficient)
        return [co.to_limbs([5] * N), co.to_limbs([7] * N), zero.copy(), zero.copy()]
    return [zero.copy() for _ in range(4)]  # "zero": every round absorbs nothing


def _device(ctx, field: int, tabs: list, prefix: bytes):
    tr = Transcript(field)
    if prefix:
        tr.append(prefix)
    sp = SumPoly([ProductPoly([tabs[0], tabs[1]], field, ctx), ProductPoly([tabs[2], tabs[3]], field, ctx)])
    p = zk_amd.gkr_prove(0, sp, tr, ctx=ctx)
    return [list(q.coefficient) for q in p.proof_polynomials], list(p.random_challenges)


def _oracle(field: int, tabs: list, prefix: bytes):
    tr = co.Transcript()
    if prefix:
        tr.append(prefix)
    polys, chal = co.gkr_prove(field, tabs, tr)
    return [list(q) for q in polys], list(chal)


@pytest.mark.parametrize("field", [0, 1, 2])
@pytest.mark.parametrize("n", [8, 9, 12, 16, 19])
def test_device_fs_matches_oracle(monkeypatch, field, n):
    tabs = _tables(field, n, "random")
    want = _oracle(field, tabs, b"")
    monkeypatch.setenv("ZK_DEVICE_FS", "1")
    for h in ("4", "0"):
        monkeypatch.setenv("ZK_HOST_ROUNDS", h)
        ctx = zk_amd.Context(0)
        try:
            ctx.reset_stats()
            assert _device(ctx, field, tabs, b"") == want, f"ZK_HOST_ROUNDS={h}"
            assert _device(ctx, field, tabs, b"") == want, f"ZK_HOST_ROUNDS={h} (second proof, same context)"
            if h == "0":
                assert ctx.stats()["device_fs_rounds"] > 0, "the device drew no challenge"
        finally:
            ctx.close()


@pytest.mark.parametrize("field", [0, 2])
@pytest.mark.parametrize("shape", ["linear", "constant", "zero"])
def test_device_fs_trimmed_absorbs(monkeypatch, field, shape):
    n = 12
    tabs = _tables(field, n, shape)
    want = _oracle(field, tabs, b"")
    expect_len = {"linear": 2, "constant": 1, "zero": 0}[shape]
    assert all(len(q) == expect_len for q in want[0][4:]), "fixture does not trim as intended"
    monkeypatch.setenv("ZK_DEVICE_FS", "1")
    monkeypatch.setenv("ZK_HOST_ROUNDS", "0")
    ctx = zk_amd.Context(0)
    try:
        ctx.reset_stats()
        assert _device(ctx, field, tabs, b"") == want
        assert ctx.stats()["device_fs_rounds"] > 0
    finally:
        ctx.close()


@pytest.mark.parametrize("plen", [1, 100, 135, 136, 137, 300])
def test_device_fs_after_caller_transcript_bytes(monkeypatch, plen):
    field, n = 0, 14
    tabs = _tables(field, n, "random")
    prefix = bytes((7 * i + 3) & 0xFF for i in range(plen))
    want = _oracle(field, tabs, prefix)
    monkeypatch.setenv("ZK_DEVICE_FS", "1")
    monkeypatch.setenv("ZK_HOST_ROUNDS", "0")
    ctx = zk_amd.Context(0)
    try:
        assert _device(ctx, field, tabs, prefix) == want
    finally:
        ctx.close()


@pytest.mark.parametrize("field", [0, 2])
def test_device_fs_default_off_same_proof(monkeypatch, field):
    """Host and device Fiat-Shamir give the same proof on one table (22 variables)."""
    n = 22
    tabs = _tables(field, n, "random")
    got = {}
    for dfs in ("0", "1"):
        monkeypatch.setenv("ZK_DEVICE_FS", dfs)
        ctx = zk_amd.Context(0)
        try:
            got[dfs] = _device(ctx, field, tabs, b"")
        finally:
            ctx.close()
    assert got["0"] == got["1"]
