"""CPU checks of the product library: it loads, exports every symbol that
include/zk_sumcheck.h declares, refuses to run compute without a GPU, and
its host-side logic (transcript, serialisation, gkr_verify) matches the oracle."""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np
import pytest

import coracle as co
import pyoracle as po
from conftest import ROOT

import zk_amd
from zk_amd import _lib
from zk_amd.elems import as_limbs, ptr, to_ints

HEADER = os.path.join(ROOT, "include", "zk_sumcheck.h")


def declared_functions() -> list[str]:
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = re.findall(r"\b(zk_[a-z0-9_]+)\s*\(", src)
    return sorted(set(n for n in names if not n.endswith("_fn")))


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    names = declared_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), f"missing export {n}"
    assert set(names) == set(_lib.SIGNATURES), "binding table out of sync with the header"


def test_abi_version():
    assert _lib.lib().zk_abi_version() == _lib.ABI_VERSION == 15


def test_nm_exports_match_header():
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (zk_[a-z0-9_]+)$", out, flags=re.M))
    assert set(declared_functions()) <= exported


def _gpu_present() -> bool:
    return os.path.exists("/dev/kfd") and bool([d for d in os.listdir("/dev/dri")] if os.path.exists("/dev/dri") else [])


@pytest.mark.skipif(_gpu_present(), reason="this host has a GPU")
def test_no_gpu_means_loud_failure():
    h = C.c_void_p()
    rc = _lib.lib().zk_ctx_create(0, C.byref(h))
    assert rc == _lib.ZK_EDEVICE
    assert b"no CPU fallback" in _lib.lib().zk_last_error() or b"device" in _lib.lib().zk_last_error()
    with pytest.raises(zk_amd.ZkError):
        zk_amd.Context(0)


# --- host logic vs oracle ------------------------------------------------------
@pytest.mark.parametrize("field", [0, 1, 2])
def test_transcript_matches_oracle(field):
    t = zk_amd.Transcript(field)
    o = po.Transcript(field)
    for chunk in [b"zero knowledge", b"", bytes(range(200)), b"\x01" * 136, b"x" * 500]:
        t.append(chunk)
        o.append(chunk)
        assert t.get_random_challenge() == o.get_random_challenge()
    t2 = t.clone()
    assert t2.get_random_challenge() == t.get_random_challenge()


@pytest.mark.parametrize("field", [0, 1, 2])
def test_fq_vec_to_bytes_matches_oracle(field):
    vals = po.synth(field, 5, 0, 0, 9) + [0, 1, po.MODULI[field] - 1]
    assert zk_amd.fq_vec_to_bytes(vals, field) == po.fq_vec_to_bytes(vals)
    with pytest.raises(ValueError):
        zk_amd.fq_vec_to_bytes([po.MODULI[field]], field)  # >= p is not a field element


def test_montgomery_repr_roundtrip_through_transcript():
    # challenge in Montgomery repr == to_mont(canonical challenge)
    L = _lib.lib()
    for f in range(3):
        ta, tb = L.zk_transcript_new(), L.zk_transcript_new()
        a, b = np.zeros((1, 4), np.uint64), np.zeros((1, 4), np.uint64)
        L.zk_transcript_get_random_challenge(ta, f, 0, ptr(a))
        L.zk_transcript_get_random_challenge(tb, f, 1, ptr(b))
        m = np.zeros((1, 4), np.uint64)
        co.lib().or_fe_to_mont(f, a.ctypes.data, m.ctypes.data)
        assert np.array_equal(m, b)
        L.zk_transcript_free(ta)
        L.zk_transcript_free(tb)


@pytest.mark.parametrize("field", [0, 1, 2])
def test_gkr_verify_matches_oracle(field, golden):
    g = golden["gkr_prove_10"][field]
    polys = [[int(c, 16) for c in p] for p in g["round_polys"]]
    claim = int(g["claimed_sum"], 16)
    res = zk_amd.gkr_verify([zk_amd.UnivariatePoly(p, field) for p in polys], claim, zk_amd.Transcript(field))
    assert res.verified and res.final_claimed_sum == int(g["final_claim"], 16)
    assert res.random_challenges == [int(c, 16) for c in g["challenges"]]
    bad = zk_amd.gkr_verify([zk_amd.UnivariatePoly(p, field) for p in polys], claim + 1, zk_amd.Transcript(field))
    assert not bad.verified and bad.final_claimed_sum == 0 and bad.random_challenges == [0]


def test_gkr_verify_reference_kat():  # sum_check_protocol.rs:247-269 via golden
    tabs = [[0, 0, 0, 2], [0, 0, 0, 3], [0, 0, 0, 2], [0, 0, 0, 3]]
    polys, cs, chal = po.gkr_prove(1, 12, tabs, po.Transcript(1))
    v = zk_amd.gkr_verify([zk_amd.UnivariatePoly(p, 1) for p in polys], cs, zk_amd.Transcript(1))
    assert v.verified and v.random_challenges == chal


def test_gkr_verify_empty_and_trimmed_polys():
    # zero round polynomial (all coefficients trimmed) is valid for claim 0
    v = zk_amd.gkr_verify([zk_amd.UnivariatePoly([], 0)], 0, zk_amd.Transcript(0))
    ok, fin, ch = po.gkr_verify(0, [[]], 0, po.Transcript(0))
    assert v.verified == ok and v.final_claimed_sum == fin and v.random_challenges == ch
    v0 = zk_amd.gkr_verify([], 5, zk_amd.Transcript(0))
    assert v0.verified and v0.final_claimed_sum == 5 and v0.random_challenges == []


def test_reference_shaped_constructors_panic_like_reference():
    with pytest.raises(ValueError):
        zk_amd.MultilinearPoly([1, 2, 3])
    with pytest.raises(ValueError):
        zk_amd.MultilinearPoly([])
    with pytest.raises(ValueError):  # ProductPoly::new's length check (composed_polynomial.rs:19-21), the panic test :157-175
        zk_amd.ProductPoly([[0, 0, 0, 3], [0, 0, 0, 4, 0, 0, 0, 4]])
    pp = zk_amd.ProductPoly([[0, 0, 0, 3]])
    with pytest.raises(ValueError):
        zk_amd.SumPoly([pp, zk_amd.ProductPoly([[1, 2], [3, 4]])])
    with pytest.raises(ValueError):  # reduce() indexes polys[1]
        zk_amd.SumPoly([zk_amd.ProductPoly([[1, 2], [3, 4]])]).gkr_tables()


def test_limbs_roundtrip():
    vals = [0, 1, (1 << 254) + 12345, (1 << 64) - 1]
    assert to_ints(as_limbs(vals)) == vals


def test_single_hip_runtime_in_process():
    """Loading the library and torch must leave exactly one libamdhip64 mapped
    (two runtimes double-free at interpreter exit, see _lib.lib())."""
    import subprocess
    import sys

    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "from zk_amd import _lib; _lib.lib(); import torch\n"
        "paths = {l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}\n"
        "print(len(paths), sorted(paths))\n"
    ) % os.path.join(ROOT, "zk-research-implementations_amd")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.startswith("1 "), out.stdout
    assert "free()" not in out.stderr and "double free" not in out.stderr, out.stderr[-2000:]


def test_kernel_kinds_match_header():
    """The ctypes zk_stats mirror is sized by KERNEL_KINDS: it must list exactly
    the header's ZK_K_* kinds, in order (a short mirror lets zk_ctx_get_stats
    write past the Python struct)."""
    text = open(HEADER).read()
    kinds = dict((m.group(1).lower(), int(m.group(2))) for m in re.finditer(r"ZK_K_([A-Z0-9_]+) = (\d+)", text))
    total = kinds.pop("kinds")
    assert total == len(_lib.KERNEL_KINDS)
    alias = {"gkr_lanes": "gkr_round_lanes"}  # header name -> mirror name
    assert [alias.get(k, k) for k in sorted(kinds, key=kinds.get)] == _lib.KERNEL_KINDS


@pytest.mark.parametrize("field", [0, 1, 2])
def test_transcript_serialize_roundtrip(field):
    """Checkpoint / resume: a transcript restored from its bytes continues
    exactly like the original and like the oracle, at every fill of the rate block."""
    o = po.Transcript(field)
    t = zk_amd.Transcript(field)
    for chunk in [b"", b"a", bytes(range(135)), b"\x07" * 136, b"y" * 137, bytes(300)]:
        t.append(chunk)
        o.append(chunk)
        state = t.to_bytes()
        assert len(state) == 352 and state[:4] == b"ZKTR"
        r = zk_amd.Transcript.from_bytes(state, field)
        assert r.to_bytes() == state
        want = o.get_random_challenge()
        assert r.get_random_challenge() == want
        assert t.get_random_challenge() == want
        assert r.to_bytes() == t.to_bytes()


def test_transcript_deserialize_rejects_malformed():
    t = zk_amd.Transcript(0)
    t.append(b"abc")
    s = bytearray(t.to_bytes())
    assert zk_amd.Transcript.from_bytes(bytes(s)).get_random_challenge() == t.clone().get_random_challenge()
    bad = [bytes(s[:-1]), bytes(s) + b"\0", b"XKTR" + bytes(s[4:]),
           bytes(s[:4]) + (2).to_bytes(4, "little") + bytes(s[8:]),
           bytes(s[:8]) + (136).to_bytes(4, "little") + bytes(s[12:]),
           bytes(s[:-1]) + b"\x01", b""]
    for b in bad:
        with pytest.raises(ValueError):
            zk_amd.Transcript.from_bytes(b)
