"""Generate tests/golden/kzg.json: the KZG commitments of BASELINE config 5 at
full size (and one smaller size), from the oracles.

The reference commits an MLE f over the Lagrange basis of fixed taus,
sum_i f_i * (eq(taus, i) * G1) (pcs/src/kzg_pcs/kzg.rs:51-53,131-144,183-212).
Since the eq weights sum to f(taus), that commitment is the single group
element f(taus) * G1, so a full-size commit is pinned by one MLE evaluation
(oracle/zk_oracle.c or_mle_evaluate, the restatement of
multilinear_polynomial_evaluation.rs:79-91) and one scalar multiplication
(oracle/kzg_oracle.py mul, the double-and-add restatement of mul_bigint).
tests/test_kzg_oracle.py pins that identity against the reference's own KZG
tests, and tests/test_gpu_kzg.py checks it at 2^14 against the naive sum.

Inputs (stored as their generator spec, not as data): the evaluations are
the synthetic table synth(BLS12-381 Fr, seed 5, table 0, i) of SURVEY.md 8(d)
(the bench's config-5 table), the taus are
[random.Random(55).randrange(r) for _ in range(nvars)] (bench.py config5).

Run: python tests/golden/make_kzg_golden.py   (~10 s)
"""
from __future__ import annotations

import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import coracle as co  # noqa: E402
import kzg_oracle as ko  # noqa: E402

FIELD = 2  # BLS12-381 Fr
SEED, TABLE, TAU_SEED = 5, 0, 55
SIZES = [22, 24]


def taus_for(nvars: int) -> list[int]:
    rng = random.Random(TAU_SEED)
    return [rng.randrange(ko.R) for _ in range(nvars)]


def fixture(nvars: int) -> dict:
    t0 = time.perf_counter()
    evals = co.synth(FIELD, SEED, TABLE, 0, 1 << nvars)
    taus = taus_for(nvars)
    v = co.evaluate(FIELD, evals, taus)
    x, y = ko.mul(v, ko.G1)
    return {
        "nvars": nvars,
        "evals": f"synth(bls12_381_fr, seed {SEED}, table {TABLE}, i) for i < 2^nvars (SURVEY.md 8(d))",
        "taus": f"[random.Random({TAU_SEED}).randrange(r) for _ in range(nvars)]",
        "mle_value": "0x%064x" % v,
        "commit_x": "0x%096x" % x,
        "commit_y": "0x%096x" % y,
        "oracle_seconds": round(time.perf_counter() - t0, 1),
    }


def main() -> None:
    out = {"_about": "KZG commitments of the config-5 MLE at full size: f(taus) * G1 from the C oracle's MLE "
                     "evaluation and kzg_oracle.mul (tests/golden/make_kzg_golden.py)"}
    for n in SIZES:
        out[f"bls12_381_fr_{n}_s{SEED}"] = fixture(n)
        print(n, out[f"bls12_381_fr_{n}_s{SEED}"]["oracle_seconds"], "s")
    with open(os.path.join(HERE, "kzg.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
