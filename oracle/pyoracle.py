"""ORACLE — TEST INFRASTRUCTURE ONLY.

Pure-Python restatement (Python big ints, small cases only) of the reference
sum-check path. It is the second, independent CPU restatement next to
oracle/zk_oracle.c: tests cross-check the two, pin both against the
reference's own known-answer tests, and tests/golden/make_golden.py uses this
module to write the committed golden vectors. Nothing in the product package
imports it.

Field elements are canonical Python ints in [0, p).
Reference files restated (paths relative to the reference root):
  fiat_shamir/src/fiat_shamir_transcript.rs:11-37       Transcript, fq_vec_to_bytes
  multilinear_polynomial/src/multilinear_polynomial_evaluation.rs:26-164
  multilinear_polynomial/src/composed_polynomial.rs:15-103
  univariate_polynomial/src/univariate_polynomial_dense.rs:14-109
  sum_check/src/sum_check_protocol.rs:25-175
Keccak-256 restates sha3 0.10.8 `Keccak256` (Keccak[c=512], pad 0x01..0x80);
its permutation is pinned by hashlib.sha3_256 (same permutation, pad 0x06) and
its padding by the public Keccak-256 vectors.
"""
from __future__ import annotations

MODULI = {
    0: 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001,  # BN254 Fr
    1: 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47,  # BN254 Fq
    2: 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,  # BLS12-381 Fr
}
FIELD_NAMES = {0: "bn254_fr", 1: "bn254_fq", 2: "bls12_381_fr"}
M64 = (1 << 64) - 1

# --------------------------------------------------------------------------
# Keccak-f[1600] / Keccak-256
# --------------------------------------------------------------------------
_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]
_ROT = [0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14]


def _rotl(x: int, s: int) -> int:
    return ((x << s) | (x >> (64 - s))) & M64 if s else x


def keccak_f1600(A: list[int]) -> None:
    for rnd in range(24):
        C = [A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20] for x in range(5)]
        D = [C[(x + 4) % 5] ^ _rotl(C[(x + 1) % 5], 1) for x in range(5)]
        for i in range(25):
            A[i] ^= D[i % 5]
        B = [0] * 25
        for x in range(5):
            for y in range(5):
                B[y + 5 * ((2 * x + 3 * y) % 5)] = _rotl(A[x + 5 * y], _ROT[x + 5 * y])
        for x in range(5):
            for y in range(5):
                A[x + 5 * y] = B[x + 5 * y] ^ ((~B[(x + 1) % 5 + 5 * y]) & B[(x + 2) % 5 + 5 * y])
        A[0] ^= _RC[rnd]


class _Sponge:
    RATE = 136

    def __init__(self, pad: int = 0x01):
        self.pad = pad
        self.reset()

    def reset(self) -> None:
        self.st = [0] * 25
        self.buf = bytearray()

    def _absorb_block(self, blk: bytes) -> None:
        for i in range(self.RATE // 8):
            self.st[i] ^= int.from_bytes(blk[8 * i: 8 * i + 8], "little")
        keccak_f1600(self.st)

    def update(self, data: bytes) -> None:
        self.buf += data
        while len(self.buf) >= self.RATE:
            self._absorb_block(bytes(self.buf[: self.RATE]))
            del self.buf[: self.RATE]

    def finalize_reset(self) -> bytes:
        blk = bytearray(self.buf) + bytearray(self.RATE - len(self.buf))
        blk[len(self.buf)] ^= self.pad
        blk[self.RATE - 1] ^= 0x80
        self._absorb_block(bytes(blk))
        out = b"".join(w.to_bytes(8, "little") for w in self.st[:4])
        self.reset()
        return out


def keccak256(data: bytes) -> bytes:
    s = _Sponge(0x01)
    s.update(data)
    return s.finalize_reset()


def sha3_256_via_permutation(data: bytes) -> bytes:
    """SHA3-256 built on the same permutation (pad 0x06) — checked against hashlib."""
    s = _Sponge(0x06)
    s.update(data)
    return s.finalize_reset()


# --------------------------------------------------------------------------
# Transcript (fiat_shamir_transcript.rs:5-37)
# --------------------------------------------------------------------------
def fq_vec_to_bytes(values: list[int]) -> bytes:
    return b"".join(int(v).to_bytes(32, "little") for v in values)


class Transcript:
    def __init__(self, field: int):
        self.p = MODULI[field]
        self.h = _Sponge(0x01)

    def append(self, preimage: bytes) -> None:
        self.h.update(preimage)

    def get_random_challenge(self) -> int:
        d = self.h.finalize_reset()
        self.append(d)
        return int.from_bytes(d, "little") % self.p  # from_le_bytes_mod_order

    def clone(self) -> "Transcript":
        t = Transcript.__new__(Transcript)
        t.p = self.p
        t.h = _Sponge(0x01)
        t.h.st = list(self.h.st)
        t.h.buf = bytearray(self.h.buf)
        return t


# --------------------------------------------------------------------------
# MultilinearPoly (multilinear_polynomial_evaluation.rs)
# --------------------------------------------------------------------------
def _nvars(n: int) -> int:
    if n == 0:
        raise ValueError("Invalid evaluations")  # 0.ilog2() panics
    k = n.bit_length() - 1
    if n != 1 << k:
        raise ValueError("Invalid evaluations")  # :29-31
    return k


def insert_bit(value: int, bit: int) -> int:  # :158-164
    high = value >> bit
    low = value & ((1 << bit) - 1)
    return high << (bit + 1) | low


def partial_evaluate(p: int, evals: list[int], bit: int, r: int) -> list[int]:  # :52-63
    n = _nvars(len(evals))
    if n == 0:
        raise ValueError("partial_evaluate on a constant")  # pair_points underflow panics
    inv = n - bit - 1
    out = []
    for v in range(1 << (n - 1)):
        a = insert_bit(v, inv)
        b = a | (1 << inv)
        out.append((evals[a] + r * (evals[b] - evals[a])) % p)
    return out


def evaluate(p: int, evals: list[int], point: list[int]) -> int:  # :79-91
    n = _nvars(len(evals))
    if len(point) != n:
        raise ValueError("Invalid number of values")
    cur = list(evals)
    for v in point:
        cur = partial_evaluate(p, cur, 0, v)
    return cur[0]


def scale(p: int, a: list[int], v: int) -> list[int]:  # :93-97
    return [x * v % p for x in a]


def binop(p: int, a: list[int], b: list[int], op: str) -> list[int]:  # impl Add/Mul/Sub :113-151 (zip)
    f = {"add": lambda x, y: x + y, "mul": lambda x, y: x * y, "sub": lambda x, y: x - y}[op]
    return [f(x, y) % p for x, y in zip(a, b)]


def tensor_add_mul(p: int, a: list[int], b: list[int], op: str) -> list[int]:  # :99-110
    if op == "add":
        return [(x + y) % p for x in a for y in b]
    return [(x * y) % p for x in a for y in b]


# --------------------------------------------------------------------------
# UnivariatePoly::interpolate (univariate_polynomial_dense.rs:48-74) — closed
# form of the same unique polynomial, trailing zeros trimmed (:14-18).
# --------------------------------------------------------------------------
def trim(c: list[int]) -> list[int]:
    c = list(c)
    while c and c[-1] == 0:
        c.pop()
    return c


def interpolate(p: int, xs: list[int], ys: list[int]) -> list[int]:
    n = len(xs)
    result = [0] * n
    for i in range(n):
        li = [1]
        denom = 1
        for j in range(n):
            if i == j:
                continue
            li = [((li[k - 1] if k > 0 else 0) - xs[j] * (li[k] if k < len(li) else 0)) % p for k in range(len(li) + 1)]
            denom = denom * (xs[i] - xs[j]) % p
        s = ys[i] * pow(denom, -1, p) % p
        for k in range(len(li)):
            result[k] = (result[k] + s * li[k]) % p
    return trim(result)


def uni_evaluate(p: int, coeffs: list[int], x: int) -> int:  # :20-26
    return sum(c * pow(x, i, p) for i, c in enumerate(coeffs)) % p


# --------------------------------------------------------------------------
# sum-check (sum_check_protocol.rs)
# --------------------------------------------------------------------------
def prove(field: int, evals: list[int]):  # :25-52
    p = MODULI[field]
    n = _nvars(len(evals))
    t = Transcript(field)
    t.append(fq_vec_to_bytes(evals))
    claimed = sum(evals) % p
    t.append(fq_vec_to_bytes([claimed]))
    polys, chal = [], []
    cur = list(evals)
    for _ in range(n):
        mid = len(cur) // 2
        rp = [sum(cur[:mid]) % p, sum(cur[mid:]) % p]  # :168-175
        t.append(fq_vec_to_bytes(rp))
        polys.append(rp)
        r = t.get_random_challenge()
        chal.append(r)
        cur = partial_evaluate(p, cur, 0, r)
    return polys, claimed, chal


def verify(field: int, evals: list[int], polys: list[list[int]], claimed: int) -> bool:  # :54-84
    p = MODULI[field]
    n = _nvars(len(evals))
    t = Transcript(field)
    t.append(fq_vec_to_bytes(evals))
    t.append(fq_vec_to_bytes([claimed]))
    expected = claimed
    chal = []
    for rp in polys:
        _nvars(len(rp))
        if sum(rp) % p != expected:
            return False
        t.append(fq_vec_to_bytes(rp))
        r = t.get_random_challenge()
        expected = (rp[0] + r * (rp[1] - rp[0])) % p
        chal.append(r)
    if len(chal) != n:
        raise ValueError("Invalid number of values")
    return expected == evaluate(p, evals, chal)


def gkr_round_poly(p: int, tables: list[list[int]]) -> list[int]:  # :152-166, degree 2
    ys = []
    for i in range(3):
        part = [partial_evaluate(p, tb, 0, i) for tb in tables]
        ys.append(sum(a * s + m * q for a, s, m, q in zip(*part)) % p)
    return interpolate(p, [0, 1, 2], ys)


def gkr_prove(field: int, claimed_sum: int, tables: list[list[int]], t: Transcript):  # :86-115
    """tables = [A, S, M, P] = SumPoly[ProductPoly[A,S], ProductPoly[M,P]]"""
    p = MODULI[field]
    n = _nvars(len(tables[0]))
    cur = [list(tb) for tb in tables]
    polys, chal = [], []
    for _ in range(n):
        rp = gkr_round_poly(p, cur)
        t.append(fq_vec_to_bytes(rp))
        polys.append(rp)
        r = t.get_random_challenge()
        chal.append(r)
        cur = [partial_evaluate(p, tb, 0, r) for tb in cur]
    return polys, claimed_sum, chal


def gkr_verify(field: int, round_polys: list[list[int]], claimed_sum: int, t: Transcript):  # :117-150
    p = MODULI[field]
    chal = []
    for rp in round_polys:
        if (uni_evaluate(p, rp, 0) + uni_evaluate(p, rp, 1)) % p != claimed_sum:
            return False, 0, [0]
        t.append(fq_vec_to_bytes(rp))
        r = t.get_random_challenge()
        chal.append(r)
        claimed_sum = uni_evaluate(p, rp, r)
    return True, claimed_sum, chal


# --------------------------------------------------------------------------
# Synthetic inputs; identical to zk_oracle.c and the device
# generator: limb k of element i of table t = splitmix64(key + 4 i + k),
# key = splitmix64(splitmix64(seed) + t); value = 256-bit LE integer mod p.
# --------------------------------------------------------------------------
def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def synth(field: int, seed: int, table: int, index0: int, count: int) -> list[int]:
    p = MODULI[field]
    key = splitmix64((splitmix64(seed) + table) & M64)
    out = []
    for i in range(index0, index0 + count):
        v = 0
        for k in range(4):
            v |= splitmix64((key + 4 * i + k) & M64) << (64 * k)
        out.append(v % p)
    return out


# ---------------------------------------------------------------------------
# Proof blob (format in include/zk_sumcheck.h "Proof blob"),
# written independently of the library's serialiser so the tests compare two
# implementations of the format. Test infrastructure only.
# ---------------------------------------------------------------------------
BLOB_GKR, BLOB_SUMCHECK = 1, 2


def proof_blob(kind: int, field: int, claimed_sum: int, round_polys: list[list[int]]) -> bytes:
    out = bytearray(b"ZKSP")
    out += bytes([1, kind, field, 0])
    out += len(round_polys).to_bytes(4, "little")
    out += fq_vec_to_bytes([claimed_sum])
    for poly in round_polys:
        out += bytes([len(poly)])
        out += fq_vec_to_bytes(list(poly))
    return bytes(out)
