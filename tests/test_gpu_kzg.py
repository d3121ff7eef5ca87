"""Multilinear KZG over BLS12-381 G1 on the GPU, through the
C ABI, against the reference-faithful restatement (oracle/kzg_oracle.py) and
the reference's own KZG tests (pcs/src/kzg_pcs/kzg.rs:214-464). With known
taus every commitment is also checked against f(taus) * G (the MLE value
times the generator: sum_i f_i eq(taus, i) = f(taus)), a size-independent
property that pins large MSMs with one scalar multiplication."""
from __future__ import annotations

import random

import pytest

import kzg_oracle as ko
import pyoracle as po

from zk_amd.kzg import KZG, msm_g1

pytestmark = pytest.mark.gpu
R = ko.R
TAUS = [5, 2, 3]
EVALS = [0, 4, 0, 4, 0, 4, 3, 7]


def test_reference_kzg_tests(ctx):  # kzg.rs:233-400
    k = KZG(TAUS, ctx)
    want = [(-8) % R, 12, 16, (-24) % R, 10, (-15) % R, (-20) % R, 30]
    assert k.lagrange_basis() == [ko.mul(x, ko.G1) for x in want]
    assert k.commit(EVALS) == ko.mul(42, ko.G1)
    point = [6, 4, 0]
    v = k.open(point, EVALS)
    assert v == 72
    assert k.get_proof(v, point, EVALS) == [ko.mul(x, ko.G1) for x in (6, 18, 4)]
    k.close()


def test_suffix_bases(ctx):
    rng = random.Random(3)
    taus = [rng.randrange(R) for _ in range(5)]
    k = KZG(taus, ctx)
    for v in range(0, 6):
        assert k.lagrange_basis(v) == ko.get_lagrange_basis(taus[5 - v:]) if v else [ko.G1]
    k.close()


@pytest.mark.parametrize("n", [1, 6])
def test_commit_equals_naive_oracle(ctx, n):
    rng = random.Random(10 + n)
    taus = [rng.randrange(R) for _ in range(n)]
    evals = [rng.randrange(R) for _ in range(1 << n)]
    k = KZG(taus, ctx)
    c = k.commit(evals)
    assert c == ko.commit(evals, ko.get_lagrange_basis(taus))
    assert c == ko.mul(po.evaluate(R, evals, taus), ko.G1)
    k.close()


def test_large_commit_equals_mle_value_times_g(ctx):
    rng = random.Random(99)
    n = 14
    taus = [rng.randrange(R) for _ in range(n)]
    evals = [rng.randrange(R) for _ in range(1 << n)]
    k = KZG(taus, ctx)
    assert k.commit(evals) == ko.mul(po.evaluate(R, evals, taus), ko.G1)
    k.close()


def test_skewed_scalars(ctx):
    rng = random.Random(5)
    n = 12
    taus = [rng.randrange(R) for _ in range(n)]
    k = KZG(taus, ctx)
    N = 1 << n
    assert k.commit([7] * N) == ko.mul(7, ko.G1)  # sum_i L_i = G
    assert k.commit([0] * N) is None
    one_hot = [0] * N
    one_hot[1234] = rng.randrange(R)
    assert k.commit(one_hot) == ko.mul(one_hot[1234] * po.evaluate(R, [int(i == 1234) for i in range(N)], taus), ko.G1)
    small = [rng.randrange(16) for _ in range(N)]
    assert k.commit(small) == ko.mul(po.evaluate(R, small, taus), ko.G1)
    assert k.commit([R - 1] * N) == ko.neg(ko.G1)
    k.close()


def test_get_proof_matches_reference_faithful_oracle(ctx):
    rng = random.Random(8)
    n = 5
    taus = [rng.randrange(R) for _ in range(n)]
    evals = [rng.randrange(R) for _ in range(1 << n)]
    point = [rng.randrange(R) for _ in range(n)]
    k = KZG(taus, ctx)
    v = k.open(point, evals)
    assert v == po.evaluate(R, evals, point)
    assert k.get_proof(v, point, evals) == ko.get_proof(evals, v, point, ko.get_lagrange_basis(taus))
    k.close()


def test_get_proof_quotients_at_taus(ctx):
    rng = random.Random(9)
    n = 12
    taus = [rng.randrange(R) for _ in range(n)]
    evals = [rng.randrange(R) for _ in range(1 << n)]
    point = [rng.randrange(R) for _ in range(n)]
    k = KZG(taus, ctx)
    v = k.open(point, evals)
    proof = k.get_proof(v, point, evals)
    cur = [(e - v) % R for e in evals]
    for i in range(n):
        q = ko.get_quotient(cur)
        assert proof[i] == ko.mul(po.evaluate(R, q, taus[i + 1:]) if len(q) > 1 else q[0], ko.G1), i
        cur = ko.get_remainder(cur, point[i])
    k.close()


def test_msm_arbitrary_bases(ctx):
    rng = random.Random(12)
    bases = [ko.mul(rng.randrange(R), ko.G1) for _ in range(100)] + [None]
    scalars = [rng.randrange(R) for _ in range(len(bases))]
    want = None
    for s, b in zip(scalars, bases):
        want = ko.add(want, ko.mul(s, b))
    assert msm_g1(bases, scalars, ctx) == want
    assert msm_g1([], [], ctx) is None


def test_msm_ragged_multi_block_signed_digits(ctx):
    """An MSM whose length is not a power of two and spans three blocks of the
    bucket sort (msm.hpp kSortPts = 16 384, the last one partial), over a few
    repeated bases (equal points meet in a bucket: the XYZZ doubling and
    cancellation cases), with scalars that hit the signed-digit edges: every
    window at 2^(c-1) (bucket 0's magnitude), every bit set (a carry through
    every window), r - 1, 0 and 1. Oracle: sum_i s_i k_i * G for bases k_i G."""
    rng = random.Random(21)
    n = 2 * 16384 + 777  # c = 12: 22 windows, 2^11 buckets each
    ks = [1, 2, 3, 5, 8, 13, 21]
    pts = [ko.mul(k, ko.G1) for k in ks]
    c = 12
    half_all = sum(1 << (c * w + c - 1) for w in range((256 + c - 1) // c)) % R
    special = [half_all, (1 << 255) - 1, R - 1, 0, 1, (1 << 11), (1 << 12) - 1]
    scalars = [rng.randrange(R) for _ in range(n)]
    for i, v in enumerate(special * 50):
        scalars[(i * 977) % n] = v % R
    bases = [pts[i % len(ks)] for i in range(n)]
    want = sum(s * ks[i % len(ks)] for i, s in enumerate(scalars)) % R
    assert msm_g1(bases, scalars, ctx) == ko.mul(want, ko.G1)
    # all one point (every entry of a window in one bucket) and a cancelling pair
    assert msm_g1([pts[0]] * 20000, [3] * 20000, ctx) == ko.mul(60000, ko.G1)
    assert msm_g1([pts[1], pts[1]], [5, R - 5], ctx) is None


def test_invalid_inputs(ctx):
    with pytest.raises(ValueError, match="not on the curve"):
        msm_g1([(1, 2)], [1], ctx)
    with pytest.raises(ValueError, match="Invalid num of vars"):
        KZG([], ctx)


def test_reference_verify_end_to_end(ctx):  # kzg.rs:402-463: setup, commit, open, get_proof on the GPU; verify
    import pairing_oracle as pao

    k = KZG([5, 2, 3], ctx)
    evals = [0, 4, 0, 4, 0, 4, 3, 7]
    point = [6, 4, 0]
    assert k.g2_taus == pao.g2_taus([5, 2, 3])
    c = k.commit(evals)
    v = k.open(point, evals)
    proof = k.get_proof(v, point, evals)
    assert KZG.verify(c, v, proof, point, k.g2_taus)
    assert not KZG.verify(c, v, [ko.G1, ko.G1, ko.G1], point, k.g2_taus)
    k.close()


def test_verify_random_12_var_opening(ctx):
    rng = random.Random(12)
    R = ko.R
    n = 12
    taus = [rng.randrange(R) for _ in range(n)]
    evals = [rng.randrange(R) for _ in range(1 << n)]
    point = [rng.randrange(R) for _ in range(n)]
    k = KZG(taus, ctx)
    c = k.commit(evals)
    v = k.open(point, evals)
    assert v == po.evaluate(R, evals, point)
    proof = k.get_proof(v, point, evals)
    g2t = k.g2_taus
    assert KZG.verify(c, v, proof, point, g2t)
    assert not KZG.verify(c, (v + 1) % R, proof, point, g2t)
    bad = list(proof)
    bad[5] = ko.add(bad[5], ko.G1)
    assert not KZG.verify(c, v, bad, point, g2t)
    k.close()


@pytest.mark.parametrize("n", [22, 24])
def test_full_size_commit_equals_mle_value_times_g(ctx, n):
    """BASELINE config 5 at full size (kzg.rs:51-53,131-144): the commitment of
    the bench's 2^n-point table through zk_dev_kzg_commit, whose window width
    grows with n (kzg.hip msm_g1_device: signed digits, c = 19 at 2^22 with
    14 windows, 20 at 2^24 with 13 windows of 2^19 buckets, the top window's
    digits small — parameters the small tests never reach), equals
    f(taus) * G1 from the C oracle's MLE evaluation, and the committed fixture
    (tests/golden/kzg.json, tests/golden/make_kzg_golden.py)."""
    import json
    import os

    import coracle as co
    import numpy as np

    from zk_amd._lib import check, lib
    from zk_amd.elems import ptr
    from zk_amd.kzg import _points

    rng = random.Random(55)  # bench.py config5 taus
    taus = [rng.randrange(R) for _ in range(n)]
    k = KZG(taus, ctx)
    evals = ctx.synth(2, 1 << n, seed=5, table=0)
    out = np.zeros((1, 12), np.uint64)
    check(lib().zk_dev_kzg_commit(ctx.h, k.h, evals.ptr, ptr(out)))
    got = _points(out)[0]
    evals.free()
    k.close()
    v = co.evaluate(2, co.synth(2, 5, 0, 0, 1 << n), taus)
    assert got == ko.mul(v, ko.G1)
    fix = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kzg.json")))[f"bls12_381_fr_{n}_s5"]
    assert got == (int(fix["commit_x"], 16), int(fix["commit_y"], 16))


def test_setup_tables_agree_across_threshold(ctx):
    """Setups below 2^16 points build their basis from the 8-bit fixed-base
    table (k_fixed_base8), larger ones from the 20-bit signed-window table that
    every context on the device shares (kzg.hip FixedBaseCache): the
    15-variable suffix basis of a 16-variable setup equals a 15-variable
    setup's basis, and a second context's 16-variable setup (cached table)
    commits to the same point."""
    import zk_amd

    rng = random.Random(16)
    taus = [rng.randrange(R) for _ in range(16)]
    k16 = KZG(taus, ctx)
    k15 = KZG(taus[1:], ctx)
    assert k16.lagrange_basis(15) == k15.lagrange_basis()
    evals = [rng.randrange(R) for _ in range(1 << 16)]
    c = k16.commit(evals)
    assert c == ko.mul(po.evaluate(R, evals, taus), ko.G1)
    ctx2 = zk_amd.Context(0)
    try:
        k2 = KZG(taus, ctx2)
        assert k2.commit(evals) == c
        k2.close()
    finally:
        ctx2.close()
    k16.close()
    k15.close()


@pytest.mark.parametrize("balanced", ["0", "1"])
def test_bucket_sum_paths_agree(monkeypatch, balanced):
    """Both bucket-sum paths (ZK_MSM_BALANCED=1, the default: equal tasks of
    kBalTask entries across bucket boundaries with XYZZ partials; 0: one task
    per <= 32 entries of a bucket) give the oracle's MSM on random scalars, on
    buckets split over many tasks (one base 20 000 times: equal partials meet
    in the XYZZ doubling), and on cancelling pairs."""
    import zk_amd

    monkeypatch.setenv("ZK_MSM_BALANCED", balanced)
    ctx = zk_amd.Context(0)
    try:
        rng = random.Random(31)
        ks = [rng.randrange(1, 1000) for _ in range(9)]
        pts = [ko.mul(k, ko.G1) for k in ks]
        n = 3 * 16384 + 5
        scalars = [rng.randrange(R) for _ in range(n)]
        bases = [pts[i % len(ks)] for i in range(n)]
        want = sum(s * ks[i % len(ks)] for i, s in enumerate(scalars)) % R
        assert msm_g1(bases, scalars, ctx) == ko.mul(want, ko.G1)
        assert msm_g1([pts[0]] * 20000, [3] * 20000, ctx) == ko.mul(60000 * ks[0], ko.G1)
        assert msm_g1([pts[2], pts[2], pts[3]], [5, R - 5, 0], ctx) is None
    finally:
        ctx.close()


@pytest.mark.parametrize("batch", ["0", None])
def test_get_proof_large_window_verifies(ctx, monkeypatch, batch):
    """KZG::get_proof (kzg.rs:59-95) at 20 variables, accepted by KZG::verify's
    pairings (kzg.rs:97-129) and rejected with a wrong opened value or a
    swapped proof. ZK_PROOF_BATCH_LEVELS=0: every quotient is its own MSM (2^19
    .. 1 points: the large signed windows, c up to 16, and the balanced bucket
    sums — the per-level path that otherwise runs only for levels of 2^20 points
    and more); default: all 20 levels in the one level-batched pass
    (msm_levels). (the per-level large-window path stays covered.)"""
    if batch is not None:
        monkeypatch.setenv("ZK_PROOF_BATCH_LEVELS", batch)
    rng = random.Random(20)
    n = 20
    taus = [rng.randrange(R) for _ in range(n)]
    evals = [rng.randrange(R) for _ in range(1 << n)]
    point = [rng.randrange(R) for _ in range(n)]
    k = KZG(taus, ctx)
    c = k.commit(evals)
    v = k.open(point, evals)
    proof = k.get_proof(v, point, evals)
    assert KZG.verify(c, v, proof, point, k.g2_taus)
    assert not KZG.verify(c, (v + 1) % R, proof, point, k.g2_taus)
    assert not KZG.verify(c, v, proof[1:] + proof[:1], point, k.g2_taus)
    k.close()


@pytest.mark.parametrize("batch", ["0", "1", "6", "14", "20"])
def test_get_proof_level_batched_quotients(ctx, monkeypatch, batch):
    """kzg_get_proof commits its last ZK_PROOF_BATCH_LEVELS quotients (20 by
    default: <= 2^19 points each) in one level-batched MSM pass (msm_levels:
    level v = points [2^v - 1, 2^(v+1) - 1) of the suffix bases, its own W
    windows); every split gives the per-level proof, and each element equals
    q_i(taus) * G1 (16 variables: two levels committed alone at 14, all
    batched at 20)."""
    rng = random.Random(31)
    n = 16
    taus = [rng.randrange(R) for _ in range(n)]
    evals = [rng.randrange(R) for _ in range(1 << n)]
    point = [rng.randrange(R) for _ in range(n)]
    k = KZG(taus, ctx)
    v = k.open(point, evals)
    monkeypatch.setenv("ZK_PROOF_BATCH_LEVELS", batch)
    proof = k.get_proof(v, point, evals)
    cur = [(e - v) % R for e in evals]
    for i in range(n):
        q = ko.get_quotient(cur)
        assert proof[i] == ko.mul(po.evaluate(R, q, taus[i + 1:]) if len(q) > 1 else q[0], ko.G1), (batch, i)
        cur = ko.get_remainder(cur, point[i])
    k.close()


@pytest.mark.parametrize("n,batch", [(3, None), (12, None), (16, "6"), (20, "0")])
def test_get_proof_device_resident_equals_host(ctx, monkeypatch, n, batch):
    """zk_dev_kzg_get_proof (evaluations already in HBM, no upload) gives the
    host entry point's proof, element for element, and KZG::verify accepts it;
    the device table is left as it was (the reference's get_proof borrows f)."""
    from zk_amd import Field

    if batch is not None:
        monkeypatch.setenv("ZK_PROOF_BATCH_LEVELS", batch)
    rng = random.Random(700 + n)
    taus = [rng.randrange(R) for _ in range(n)]
    evals = [rng.randrange(R) for _ in range(1 << n)] if n > 3 else EVALS
    point = [rng.randrange(R) for _ in range(n)]
    k = KZG(taus, ctx)
    v = k.open(point, evals)
    t = ctx.upload(Field.BLS12_381_FR, evals)
    try:
        dev = k.get_proof_device(v, point, t)
        assert dev == k.get_proof(v, point, evals)
        assert KZG.verify(k.commit(evals), v, dev, point, k.g2_taus)
        assert t.to_ints() == evals
        with pytest.raises(ValueError):
            k.get_proof_device(v, point, ctx.upload(Field.BLS12_381_FR, evals[: len(evals) // 2]))
    finally:
        t.free()
        k.close()


def test_release_fixed_base_cache_rebuilds(ctx):
    """zk_kzg_release_fixed_base_cache (the 654 MB table large setups
    share is no longer pinned for the process): after a release, the next
    2^16-point setup rebuilds it and gives the same basis; releasing twice, or
    a device with no table, is a no-op."""
    from zk_amd.kzg import release_fixed_base_cache

    rng = random.Random(16)
    taus = [rng.randrange(R) for _ in range(16)]
    evals = [rng.randrange(R) for _ in range(1 << 16)]
    k = KZG(taus, ctx)
    c0 = k.commit(evals)
    k.close()
    release_fixed_base_cache()
    release_fixed_base_cache(0)
    k = KZG(taus, ctx)
    assert k.commit(evals) == c0 == ko.mul(po.evaluate(R, evals, taus), ko.G1)
    k.close()
