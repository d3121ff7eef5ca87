"""Pre-enqueued rounds (default): every round kernel is enqueued before round
0's sums are read and waits in-kernel for the host to post its challenge.

* The proof is identical with and without pre-enqueue (ZK_PRELAUNCH=0 launches
  each round after its challenge), and equal to the oracle's.
* From round 2 on two rounds run per kernel (k_gkr_dround, default); the
  proof is identical with one round per kernel (ZK_DROUND=0), for odd and
  even round counts, pre-enqueued or not. With ZK_D0=1 (default) even counts
  below 11 (or ZK_D0T=0) run rounds 0 and 1 in one pass over the inputs
  (k_gkr_d0m); the proof is identical to ZK_D0=0 (round 0, then round 1).
* The small double steps run in one persistent kernel (k_gkr_dtail, default);
  the proof is identical with one launch per step (ZK_DTAIL=0), when it
  starts at the first double step over large tables (ZK_DTAIL_MAX_QUADS) and
  with one block (ZK_DTAIL_BLOCKS=1).
* With ZK_DROUND=0 the small rounds run in one persistent kernel (k_gkr_tail);
  the proof is identical with one launch per round (ZK_TAIL=0) and when the
  tail starts at round 1 over large tables (ZK_LANES_MAX_PAIRS).
* The last ZK_HOST_ROUNDS rounds (default 4) run on the host from the tables
  the persistent tail hands over; every setting gives the oracle's proof.
* When the host fails mid-proof (here: the host all-reduce callback raises in
  round 3), the call returns ZK_ECOMM promptly — the guard releases every
  kernel still waiting instead of letting each run into its 1 s limit — and
  the same context proves correctly afterwards.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np
import pytest

import coracle as co

import zk_amd
from zk_amd._lib import ZK_ECOMM, ZkError, check, lib
from zk_amd.elems import as_limbs, ptr, to_ints

pytestmark = pytest.mark.gpu


def _prove(ctx, field: int, n: int) -> tuple[list, list]:
    tabs = [ctx.synth(field, 1 << n, seed=23, table=t) for t in range(4)]
    arr = (C.c_void_p * 4)(*[t.ptr.value for t in tabs])
    coeffs = np.zeros((n, 3, 4), np.uint64)
    nco = np.zeros(n, np.uint8)
    ch = np.zeros((n, 4), np.uint64)
    tr = zk_amd.Transcript(field)
    check(lib().zk_dev_gkr_sumcheck_prove_sharded(ctx.h, field, arr, n, 0, ptr(as_limbs([0])), tr.h, ptr(coeffs),
                                                  ptr(nco), ptr(ch)))
    return [to_ints(coeffs[k, : nco[k]]) for k in range(n)], to_ints(ch)


def _oracle(field: int, n: int) -> tuple[list, list]:
    tabs = [co.synth(field, 23, t, 0, 1 << n) for t in range(4)]
    polys, chal = co.gkr_prove(field, tabs, co.Transcript())
    return [list(p) for p in polys], list(chal)


@pytest.mark.parametrize("field", [0, 2])
def test_prelaunch_and_per_round_launch_agree(monkeypatch, field):
    n = 16
    want = _oracle(field, n)
    for mode in ("1", "0"):
        monkeypatch.setenv("ZK_PRELAUNCH", mode)
        ctx = zk_amd.Context(0)
        try:
            assert _prove(ctx, field, n) == want, f"ZK_PRELAUNCH={mode}"
        finally:
            ctx.close()


@pytest.mark.parametrize("field", [0, 1, 2])
@pytest.mark.parametrize("tail,lanes_max", [("1", None), ("0", None), ("1", str(1 << 20)), ("1", "4")])
def test_tail_kernel_modes_agree(monkeypatch, field, tail, lanes_max):
    n = 17 if lanes_max is None else 21
    want = _oracle(field, n) if n == 17 else None
    monkeypatch.setenv("ZK_DROUND", "0")
    monkeypatch.setenv("ZK_TAIL", tail)
    if lanes_max is not None:
        monkeypatch.setenv("ZK_LANES_MAX_PAIRS", lanes_max)
    ctx = zk_amd.Context(0)
    try:
        got = _prove(ctx, field, n)
        if want is None:  # compare with the per-round launches of the same context settings
            monkeypatch.setenv("ZK_TAIL", "0")
            ref = zk_amd.Context(0)
            try:
                want = _prove(ref, field, n)
            finally:
                ref.close()
        assert got == want
        assert _prove(ctx, field, n) == want  # reused tail buffer and relay slots
    finally:
        ctx.close()


@pytest.mark.parametrize("field", [0, 1, 2])
@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 9, 12, 15])
def test_double_rounds_match_oracle(monkeypatch, field, n):
    want = _oracle(field, n)
    for pre in ("1", "0"):
        monkeypatch.setenv("ZK_PRELAUNCH", pre)
        ctx = zk_amd.Context(0)
        try:
            assert _prove(ctx, field, n) == want, f"ZK_PRELAUNCH={pre}"
        finally:
            ctx.close()


@pytest.mark.parametrize("field", [0, 2])
def test_double_and_single_rounds_agree_20var(monkeypatch, field):
    n = 20
    got = {}
    for dr in ("1", "0"):
        monkeypatch.setenv("ZK_DROUND", dr)
        ctx = zk_amd.Context(0)
        try:
            got[dr] = _prove(ctx, field, n)
        finally:
            ctx.close()
    assert got["1"] == got["0"]


@pytest.mark.parametrize("field", [0, 1, 2])
@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_first_double_step_matches_oracle(monkeypatch, field, n):
    """With ZK_D0=1 even variable counts start with rounds 0 and 1 in one pass
    over the inputs (k_gkr_d0m: nine product sums on the matrix cores, nothing
    written); ZK_D0=0 runs round 0 alone and round 1 as a single step. Both
    equal the oracle, pre-enqueued and per-round launched."""
    want = _oracle(field, n)
    monkeypatch.setenv("ZK_D0T", "0")  # the two-round first pass (n >= 11 default to three rounds)
    for d0 in ("1", "0"):
        for pre in ("1", "0"):
            monkeypatch.setenv("ZK_D0", d0)
            monkeypatch.setenv("ZK_PRELAUNCH", pre)
            ctx = zk_amd.Context(0)
            try:
                assert _prove(ctx, field, n) == want, f"ZK_D0={d0} ZK_PRELAUNCH={pre}"
            finally:
                ctx.close()


@pytest.mark.parametrize("field", [0, 2])
def test_first_double_step_agrees_22var(monkeypatch, field):
    n = 22
    got = {}
    monkeypatch.setenv("ZK_D0T", "0")
    for d0 in ("1", "0"):
        monkeypatch.setenv("ZK_D0", d0)
        ctx = zk_amd.Context(0)
        try:
            got[d0] = _prove(ctx, field, n)
        finally:
            ctx.close()
    assert got["1"] == got["0"]


@pytest.mark.parametrize("field", [0, 2])
@pytest.mark.parametrize("env", [{"ZK_DTAIL": "0"}, {"ZK_DTAIL_MAX_QUADS": str(1 << 16)}, {"ZK_DTAIL_BLOCKS": "1"},
                                 {"ZK_DTAIL_MAX_QUADS": "16"}])
@pytest.mark.parametrize("n", [16, 17])
def test_dtail_modes_agree(monkeypatch, field, env, n):
    want = _oracle(field, n)
    for key, val in env.items():
        monkeypatch.setenv(key, val)
    ctx = zk_amd.Context(0)
    try:
        assert _prove(ctx, field, n) == want
        assert _prove(ctx, field, n) == want  # reused tail buffer and relay slots
    finally:
        ctx.close()


def test_host_failure_mid_proof_releases_waiting_rounds(monkeypatch):
    monkeypatch.setenv("ZK_FORCE_COLLECTIVES", "1")  # route every round through the host all-reduce at world 1
    ctx = zk_amd.Context(0)
    try:
        calls = {"n": 0}

        def failing(buf):  # identity at world 1, raises in round 3
            calls["n"] += 1
            if calls["n"] == 4:
                raise RuntimeError("peer lost")

        ctx.attach_host_comm(0, 1, failing)
        t0 = time.perf_counter()
        with pytest.raises(ZkError) as e:
            _prove(ctx, 0, 18)
        elapsed = time.perf_counter() - t0
        assert e.value.code == ZK_ECOMM
        assert elapsed < 0.5, f"waiting rounds were not released ({elapsed:.2f} s)"
        ctx.attach_host_comm(0, 1, lambda buf: None)
        assert _prove(ctx, 0, 14) == _oracle(0, 14)
    finally:
        ctx.close()


@pytest.mark.parametrize("field", [0, 1, 2])
@pytest.mark.parametrize("n", [10, 13, 16])
def test_matrix_core_double_steps_match_oracle(monkeypatch, field, n):
    """Double steps with two pending challenges on the matrix cores (k_gkr_dm,
    mfma.hpp: fold by (ra, rb) as a K = 96 int8 MFMA + REDC, grid-point
    products as K = 64 MFMAs) give the oracle's proof; ZK_DM_MIN_QUADS=64 puts
    every double step with >= 64 quads on it (n = 13: after round 0 and a
    single round, so its first double step has one pending challenge and
    stays on k_gkr_dround)."""
    want = _oracle(field, n)
    monkeypatch.setenv("ZK_DM_MIN_QUADS", "64")
    monkeypatch.setenv("ZK_D0T", "0")
    for dm in ("1", "0"):
        for pre in ("1", "0"):
            monkeypatch.setenv("ZK_DM", dm)
            monkeypatch.setenv("ZK_PRELAUNCH", pre)
            ctx = zk_amd.Context(0)
            try:
                assert _prove(ctx, field, n) == want, f"ZK_DM={dm} ZK_PRELAUNCH={pre}"
            finally:
                ctx.close()


@pytest.mark.parametrize("field", [0, 2])
def test_matrix_core_double_steps_agree_22var(monkeypatch, field):
    n = 22
    got = {}
    monkeypatch.setenv("ZK_D0T", "0")
    for dm in ("1", "0"):
        monkeypatch.setenv("ZK_DM", dm)
        ctx = zk_amd.Context(0)
        try:
            got[dm] = _prove(ctx, field, n)
        finally:
            ctx.close()
    assert got["1"] == got["0"]


@pytest.mark.parametrize("field", [0, 1, 2])
@pytest.mark.parametrize("n", [11, 12, 13, 14, 15, 16, 17, 18, 19, 20])
def test_three_round_first_pass_matches_oracle(monkeypatch, field, n):
    """Three rounds per pass (host.hpp gkr_phase): rounds 0-2 over the inputs
    (k_gkr_d0t: 27 moment tiles of corner-pair products on the matrix cores);
    triple steps that fold by the three pending challenges (eq weights,
    K = 256) and sum three rounds as 27 moment tiles (k_gkr_t33); one
    two-round step folding by three (k_gkr_dm3); double steps. ZK_D0T=0 keeps
    the two-round schedule. Both give the oracle's proof, pre-enqueued or not."""
    want = _oracle(field, n)
    for d0t in ("1", "0"):
        for pre in ("1", "0"):
            monkeypatch.setenv("ZK_D0T", d0t)
            monkeypatch.setenv("ZK_PRELAUNCH", pre)
            ctx = zk_amd.Context(0)
            try:
                assert _prove(ctx, field, n) == want, f"ZK_D0T={d0t} ZK_PRELAUNCH={pre}"
            finally:
                ctx.close()


@pytest.mark.parametrize("field", [0, 2])
@pytest.mark.parametrize("n", [23, 24])
def test_three_round_first_pass_agrees_large(monkeypatch, field, n):
    got = {}
    for d0t in ("1", "0"):
        monkeypatch.setenv("ZK_D0T", d0t)
        ctx = zk_amd.Context(0)
        try:
            got[d0t] = _prove(ctx, field, n)
        finally:
            ctx.close()
    assert got["1"] == got["0"]


@pytest.mark.parametrize("field", [0, 1, 2])
@pytest.mark.parametrize("n", [8, 10, 12, 15, 16, 19])
def test_host_rounds_match_oracle(monkeypatch, field, n):
    """The last ZK_HOST_ROUNDS rounds on the host (host.hpp "host rounds"): the
    persistent tail's last device step stores its output tables word-major to
    pinned host memory (kernels.hpp st_fe_sys) and the host folds them by that
    step's challenges and runs the remaining rounds. Every H (0 = all on the
    device; odd H rounds down; H larger than the schedule allows falls back to
    the device) gives the oracle's proof, twice on one context (the host
    table buffer is reused)."""
    want = _oracle(field, n)
    for h in ("0", "2", "4", "5", "6", "8", "40"):
        monkeypatch.setenv("ZK_HOST_ROUNDS", h)
        ctx = zk_amd.Context(0)
        try:
            assert _prove(ctx, field, n) == want, f"ZK_HOST_ROUNDS={h}"
            assert _prove(ctx, field, n) == want, f"ZK_HOST_ROUNDS={h} (second proof)"
        finally:
            ctx.close()
