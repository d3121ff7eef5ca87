"""Median wall time of the circuit GKR prover (bench.py gkr_circuit's workload)
for several ZK_CIRCUIT_HOST_LGL splits, alternating, in one process. Diagnostic."""
import os
import random
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zk-research-implementations_amd"))
import torch  # noqa: F401,E402  (one HIP runtime: torch first)
import zk_amd  # noqa: E402
from zk_amd.gkr import Circuit, Operation, prove, verify  # noqa: E402

log_inputs = int(sys.argv[1]) if len(sys.argv) > 1 else 12
splits = [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["8"])]
rng = random.Random(11)
structure = [[rng.choice((Operation.Add, Operation.Mul)) for _ in range(1 << (log_inputs - 1 - i))]
             for i in range(log_inputs)]
inputs = [rng.randrange(zk_amd.modulus(0)) for _ in range(1 << log_inputs)]
circ = Circuit(structure, 0)
ctxs = {}
for s in splits:
    os.environ["ZK_CIRCUIT_HOST_LGL"] = str(s)
    ctxs[s] = zk_amd.Context(0)
    pr = prove(circ, inputs, ctxs[s])
    assert verify(pr, circ, inputs)
times = {s: [] for s in splits}
ref = None
for it in range(5):
    for s in splits:
        for _ in range(5):
            t0 = time.perf_counter()
            pr = prove(circ, inputs, ctxs[s])
            times[s].append(time.perf_counter() - t0)
        if ref is None:
            ref = pr.random_challenges
        assert pr.random_challenges == ref
for s in splits:
    t = sorted(times[s])
    print(f"host_lgl {s}: median {t[len(t) // 2] * 1e3:.3f} ms, min {t[0] * 1e3:.3f} ms ({len(t)} proofs)", flush=True)
for c in ctxs.values():
    c.close()
