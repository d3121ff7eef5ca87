"""Generate tests/golden/large.json: the GKR sum-check proofs of the BASELINE
workloads at their full sizes (BASELINE.json configs 3, 4, 5 and the bench's
multi-GPU headline sizes), from the C oracle.

Each proof comes from `or_gkr_prove_fast` (oracle/zk_oracle.c: the fused
OpenMP restatement of gkr_prove, sum_check_protocol.rs:86-115 with
get_round_partial_polynomial_proof_gkr :152-166). That restatement gives the
same transcript as the reference-faithful `or_gkr_prove` — asserted here on a
16-variable case before anything is written, and in tests/test_oracle.py on the
golden 10-variable vectors. Tables are the counter-based synthetic inputs of
SURVEY.md 8(d) (stored as their generator spec, not as data).

Per workload the file holds the round polynomials, the challenges, the true
claimed sum (round 0's s(0) + s(1)) and the Keccak-256 digest of the proof
blob (include/zk_sumcheck.h "Proof blob"; written by the oracle's independent
writer, oracle/pyoracle.py proof_blob). Fiat-Shamir challenge values are
pinned by the restated specification and the public Keccak vectors, not by
reference outputs (the reference never asserts a challenge).

Run: python tests/golden/make_large_golden.py   (~1-2 min on 8 cores, ~35 GiB
peak for the 27-variable case; --max-nvars 26 skips it)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import coracle as co  # noqa: E402
import pyoracle as po  # noqa: E402

# (key, field, nvars, seed, what)
WORKLOADS = [
    ("bn254_fr_24_s3", 0, 24, 3, "BASELINE config 3 (bench headline, 1 GPU)"),
    ("bls12_381_fr_24_s5", 2, 24, 5, "BASELINE config 5 (second modulus)"),
    ("bn254_fr_26_s4", 0, 26, 4, "BASELINE config 4 (26 variables in total, any GPU count)"),
    ("bn254_fr_23_s3", 0, 23, 3, "odd variable count (d0t, t33 x2, dm3 at an odd level)"),
    ("bn254_fr_25_s3", 0, 25, 3, "bench headline at 2 GPUs (24 variables per GPU)"),
    ("bn254_fr_26_s3", 0, 26, 3, "bench headline at 4 GPUs"),
    ("bn254_fr_27_s3", 0, 27, 3, "bench headline at 8 GPUs"),
]


def hx(v: int) -> str:
    return "0x%064x" % v


def gkr_fixture(field: int, n: int, seed: int) -> dict:
    t0 = time.perf_counter()
    tabs = [co.synth(field, seed, t, 0, 1 << n) for t in range(4)]
    polys, chal = co.gkr_prove(field, tabs, co.Transcript(), fast=True)
    del tabs
    p = po.MODULI[field]
    c0 = polys[0]
    claimed = (po.uni_evaluate(p, c0, 0) + po.uni_evaluate(p, c0, 1)) % p  # s_0(0) + s_0(1) = sum of A S + M P
    blob = po.proof_blob(po.BLOB_GKR, field, claimed, polys)
    ok, _, ch2 = po.gkr_verify(field, polys, claimed, po.Transcript(field))
    assert ok and ch2 == chal, "oracle proof does not verify"
    return {
        "field": field,
        "nvars": n,
        "seed": seed,
        "tables": "synth(field, seed, table t = 0..3 (A, S, M, P), index i) for i < 2^nvars (SURVEY.md 8(d))",
        "claimed_sum": hx(claimed),
        "round_polys": [[hx(c) for c in poly] for poly in polys],
        "challenges": [hx(c) for c in chal],
        "blob_keccak256": po.keccak256(blob).hex(),
        "oracle_seconds": round(time.perf_counter() - t0, 1),
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-nvars", type=int, default=27)
    args = ap.parse_args()
    # the fused restatement equals the reference-faithful one (here: 16 vars, every field)
    for f in range(3):
        tabs = [co.synth(f, 41, t, 0, 1 << 16) for t in range(4)]
        assert co.gkr_prove(f, tabs, co.Transcript(), fast=True) == co.gkr_prove(f, tabs, co.Transcript())
    path = os.path.join(HERE, "large.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    out["_about"] = ("GKR sum-check proofs of the BASELINE workloads at full size from oracle/zk_oracle.c "
                     "or_gkr_prove_fast (tests/golden/make_large_golden.py); threads: %d" % co.threads())
    for key, field, n, seed, what in WORKLOADS:
        if n > args.max_nvars:
            continue
        g = gkr_fixture(field, n, seed)
        g["what"] = what
        out[key] = g
        print(f"{key}: {g['oracle_seconds']} s, blob keccak {g['blob_keccak256'][:16]}", flush=True)
        with open(path, "w") as fh:
            json.dump(out, fh, indent=1)
            fh.write("\n")


if __name__ == "__main__":
    main()
