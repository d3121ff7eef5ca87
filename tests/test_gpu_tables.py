"""GPU parity of the table builders either side of the sum-check
(multilinear_polynomial_evaluation.rs:93-151): scale, element-wise Add / Mul /
Sub (zip semantics), tensor_add_mul_polynomials — host API and device-resident
— against the oracle (pyoracle.scale / binop / tensor_add_mul) and the
reference's tensor KATs (gkr_protocol.rs:362-420). Bit-exact. The device tensor
then builds the GKR-shaped S = w (+) w, P = w (x) w tables in
HBM and the proof over them matches the oracle's."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import coracle as co
import pyoracle as po

import zk_amd
from zk_amd import Field, MultilinearPoly, ProductPoly, SumPoly, Transcript
from zk_amd._lib import check, lib
from zk_amd.api import MLE_ADD, MLE_MUL, MLE_SUB
from zk_amd.elems import as_limbs, ptr, to_ints

pytestmark = pytest.mark.gpu
FIELDS = [0, 1, 2]


def _vals(field, seed, n):
    return to_ints(co.synth(field, seed, 0, 0, n))


def test_kat_tensor_add_mul(ctx):  # gkr_protocol.rs:362-420 (the reference's tensor tests)
    T = MultilinearPoly.tensor_add_mul_polynomials
    f = Field.BN254_FQ
    assert T([0, 2], [0, 3], "add", f, ctx).evaluation == [0, 3, 2, 5]
    assert T([0, 3], [0, 0, 0, 2], "add", f, ctx).evaluation == [0, 0, 0, 2, 3, 3, 3, 5]
    assert T([0, 2], [0, 3], "mul", f, ctx).evaluation == [0, 0, 0, 6]
    assert T([0, 3], [0, 0, 0, 2], "mul", f, ctx).evaluation == [0] * 7 + [6]


@pytest.mark.parametrize("field", FIELDS)
@pytest.mark.parametrize("na,nb", [(1, 1), (1, 64), (64, 1), (2, 512), (256, 256), (4096, 8)])
@pytest.mark.parametrize("op", ["add", "mul"])
def test_tensor_vs_oracle(ctx, field, na, nb, op):
    a, b = _vals(field, 11, na), _vals(field, 12, nb)
    got = MultilinearPoly.tensor_add_mul_polynomials(a, b, op, field, ctx).evaluation
    assert got == po.tensor_add_mul(po.MODULI[field], a, b, op)


def test_tensor_rejects_like_reference(ctx):
    T = MultilinearPoly.tensor_add_mul_polynomials
    with pytest.raises(ValueError):
        T([1, 2, 3], [1], "add", 0, ctx)  # length 3: MultilinearPoly::new panics
    with pytest.raises(ValueError):
        T([], [1, 2], "mul", 0, ctx)  # empty: ilog2(0) panics
    with pytest.raises(ValueError):
        T([1, 2], [1, 2], MLE_SUB, 0, ctx)  # Operation has Add and Mul only


@pytest.mark.parametrize("field", FIELDS)
@pytest.mark.parametrize("na,nb", [(1, 1), (8, 8), (1024, 16), (2, 4096)])
def test_binop_vs_oracle_zip(ctx, field, na, nb):
    a, b = _vals(field, 21, na), _vals(field, 22, nb)
    pa, pb = MultilinearPoly(a, field, ctx), MultilinearPoly(b, field, ctx)
    p = po.MODULI[field]
    assert (pa + pb).evaluation == po.binop(p, a, b, "add")
    assert (pa * pb).evaluation == po.binop(p, a, b, "mul")
    assert (pa - pb).evaluation == po.binop(p, a, b, "sub")
    assert (pb - pa).evaluation == po.binop(p, b, a, "sub")


@pytest.mark.parametrize("field", FIELDS)
@pytest.mark.parametrize("n", [0, 1, 13])
def test_scale_vs_oracle(ctx, field, n):
    a = _vals(field, 31, 1 << n)
    p = po.MODULI[field]
    for v in (0, 1, p - 1, _vals(field, 32, 1)[0]):
        assert MultilinearPoly(a, field, ctx).scale(v).evaluation == po.scale(p, a, v)


def test_reduce_like_reference(ctx):  # composed_polynomial.rs:52-54, 88-99
    f = 0
    p = po.MODULI[f]
    t = [_vals(f, 40 + i, 16) for i in range(4)]
    sp = SumPoly([ProductPoly([t[0], t[1]], f, ctx), ProductPoly([t[2], t[3]], f, ctx)])
    want = [(a * s + m * q) % p for a, s, m, q in zip(*t)]
    assert sp.reduce() == want
    assert sp.polys[0].reduce() == po.binop(p, t[0], t[1], "mul")


@pytest.mark.parametrize("field", FIELDS)
def test_device_tensor_builds_gkr_shaped_tables(ctx, field):
    """S = w (+) w and P = w (x) w over 2^(2h) entries built in HBM by
    zk_dev_mle_tensor, A and M synthetic; the device proof over them equals the
    oracle's proof over the oracle-built tables."""
    h = 6
    n = 2 * h
    w = ctx.synth(field, 1 << h, seed=50, table=0)
    S, P = ctx.alloc(field, 1 << n), ctx.alloc(field, 1 << n)
    check(lib().zk_dev_mle_tensor(ctx.h, field, MLE_ADD, w.ptr, 1 << h, w.ptr, 1 << h, S.ptr))
    check(lib().zk_dev_mle_tensor(ctx.h, field, MLE_MUL, w.ptr, 1 << h, w.ptr, 1 << h, P.ptr))
    p = po.MODULI[field]
    wv = w.to_ints()
    assert S.to_ints() == po.tensor_add_mul(p, wv, wv, "add")
    assert P.to_ints() == po.tensor_add_mul(p, wv, wv, "mul")
    A = ctx.synth(field, 1 << n, seed=51, table=1)
    M = ctx.synth(field, 1 << n, seed=51, table=2)
    dev = [A, S, M, P]
    arr = (C.c_void_p * 4)(*[d.ptr.value for d in dev])
    coeffs = np.zeros((n, 3, 4), np.uint64)
    nco = np.zeros(n, np.uint8)
    ch = np.zeros((n, 4), np.uint64)
    tr = Transcript(field)
    check(lib().zk_dev_gkr_sumcheck_prove(ctx.h, field, arr, n, 0, ptr(as_limbs([0])), tr.h, ptr(coeffs), ptr(nco),
                                          ptr(ch)))
    tabs = [d.download() for d in dev]
    polys, chal = co.gkr_prove(field, tabs, co.Transcript())
    assert [to_ints(coeffs[k, : nco[k]]) for k in range(n)] == polys
    assert to_ints(ch) == chal


def test_device_tensor_rejects_alias_and_bad_sizes(ctx):
    w = ctx.synth(0, 8, seed=1, table=0)
    out = ctx.alloc(0, 64)
    with pytest.raises(zk_amd.ZkError):
        check(lib().zk_dev_mle_tensor(ctx.h, 0, MLE_ADD, w.ptr, 8, w.ptr, 8, w.ptr))
    with pytest.raises(zk_amd.ZkError):
        check(lib().zk_dev_mle_tensor(ctx.h, 0, MLE_MUL, w.ptr, 3, w.ptr, 8, out.ptr))
