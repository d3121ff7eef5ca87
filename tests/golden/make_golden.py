"""Generate the committed golden vectors in tests/golden/*.json.

Inputs and expected outputs come from the pure-Python oracle
(oracle/pyoracle.py), cross-checked against the C oracle (oracle/zk_oracle.c)
before anything is written. The reference (Rust, arkworks) cannot be built in
this environment, so challenge values and proof bytes are
pinned by the restated algorithm + the public Keccak-256 vectors + the
reference's own known-answer tests (all asserted in tests/test_oracle.py).

Large tables are stored as (generator spec, SHA-256 of their canonical bytes),
not as data. Run: python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import coracle as co  # noqa: E402
import pyoracle as po  # noqa: E402


def hx(v: int) -> str:
    return "0x%064x" % v


def table_digest(values) -> str:
    return hashlib.sha256(po.fq_vec_to_bytes(values)).hexdigest()


def synth_spec(field, seed, table, n):
    vals = po.synth(field, seed, table, 0, 1 << n)
    return {"field": field, "seed": seed, "table": table, "nvars": n, "sha256": table_digest(vals)}, vals


def main() -> None:
    out = {}
    # --- public Keccak-256 vectors + transcript challenges --------------------
    out["keccak256"] = [
        {"msg_hex": "", "digest": po.keccak256(b"").hex()},
        {"msg_hex": b"abc".hex(), "digest": po.keccak256(b"abc").hex()},
        {"msg_hex": bytes(range(200)).hex(), "digest": po.keccak256(bytes(range(200))).hex()},
    ]
    assert out["keccak256"][0]["digest"] == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
    assert out["keccak256"][1]["digest"] == "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45"
    ch = []
    for f in range(3):
        t = po.Transcript(f)
        t.append(b"zero knowledge")  # fiat_shamir_transcript.rs:44-52 (it_hashes)
        c1 = t.get_random_challenge()
        c2 = t.get_random_challenge()
        t2 = co.Transcript()
        t2.append(b"zero knowledge")
        assert [t2.get_random_challenge(f), t2.get_random_challenge(f)] == [c1, c2]
        ch.append({"field": f, "preimage": "zero knowledge", "challenges": [hx(c1), hx(c2)]})
    out["transcript"] = ch

    # --- plain sum-check, 12-var random (BASELINE config 1), all fields -------
    sc = []
    for f in range(3):
        spec, vals = synth_spec(f, 1, 0, 12)
        polys, claimed, chal = po.prove(f, vals)
        rp, cc = co.prove(f, co.to_limbs(vals))
        assert cc == claimed and [co.from_limbs(x) for x in rp] == polys
        sc.append({"input": spec, "claimed_sum": hx(claimed), "round_polys": [[hx(a), hx(b)] for a, b in polys],
                   "challenges": [hx(c) for c in chal]})
    out["sumcheck_prove_12"] = sc

    # --- reference test_valid_proving_and_verification: 20-var constant 10 ---
    # (sum_check_protocol.rs:194-204). Table hashing is 32 MiB -> C oracle;
    # the round polys are structurally [10*2^(n-1-k)] x 2.
    import numpy as np

    n = 20
    ev = np.zeros((1 << n, 4), np.uint64)
    ev[:, 0] = 10
    rp, cc = co.prove(1, ev)
    polys = [co.from_limbs(x) for x in rp]
    assert cc == 10 << n and all(p == [10 << (n - 1 - k)] * 2 for k, p in enumerate(polys))
    # challenges: replay the transcript with the C oracle (same byte stream)
    t = co.Transcript()
    t.append(po.fq_vec_to_bytes([10]) * (1 << n))
    t.append(po.fq_vec_to_bytes([cc]))
    chal = []
    for p in polys:
        t.append(po.fq_vec_to_bytes(p))
        chal.append(t.get_random_challenge(1))
    out["sumcheck_const10_20"] = {"field": 1, "nvars": n, "value": 10, "claimed_sum": hx(cc),
                                  "challenges": [hx(c) for c in chal]}

    # --- GKR sum-check ---------------------------------------------------------
    # reference test_gkr_prover_and_verifier (sum_check_protocol.rs:247-269), BN254 Fq
    tabs = [[0, 0, 0, 2], [0, 0, 0, 3], [0, 0, 0, 2], [0, 0, 0, 3]]
    t = po.Transcript(1)
    polys, cs, chal = po.gkr_prove(1, 12, tabs, t)
    out["gkr_ref_2var"] = {"field": 1, "tables": tabs, "claimed_sum": 12,
                           "round_polys": [[hx(c) for c in p] for p in polys], "challenges": [hx(c) for c in chal]}
    # random 10-var for all three fields (GKR-shaped tables A,S,M,P, seed 3)
    g = []
    for f in range(3):
        specs, tv = zip(*[synth_spec(f, 3, k, 10) for k in range(4)])
        t = po.Transcript(f)
        polys, _, chal = po.gkr_prove(f, 0, list(tv), t)
        t2 = co.Transcript()
        polys2, chal2 = co.gkr_prove(f, [co.to_limbs(x) for x in tv], t2)
        assert polys == polys2 and chal == chal2
        P = po.MODULI[f]
        claim = (po.uni_evaluate(P, polys[0], 0) + po.uni_evaluate(P, polys[0], 1)) % P
        ok, fin, _ = po.gkr_verify(f, polys, claim, po.Transcript(f))
        assert ok
        g.append({"inputs": list(specs), "claimed_sum": hx(claim), "final_claim": hx(fin),
                  "round_polys": [[hx(c) for c in p] for p in polys], "challenges": [hx(c) for c in chal]})
    out["gkr_prove_10"] = g

    # --- fold / evaluate vectors (20-var BN254 Fr config 2, by digest) -------
    spec, _ = synth_spec(0, 2, 0, 20)
    r = po.synth(0, 2, 99, 0, 1)[0]
    folded = co.partial_evaluate(0, co.synth(0, 2, 0, 0, 1 << 20), 0, r)
    out["fold_20"] = {"input": spec, "r": hx(r),
                      "output_sha256": hashlib.sha256(folded.astype("<u8").tobytes()).hexdigest()}

    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
