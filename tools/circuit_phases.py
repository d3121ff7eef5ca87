"""Per-layer timing of the circuit GKR prover (run with ZK_DEBUG_CIRCUIT=1;
the library prints one line per layer on stderr). Diagnostic only."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zk-research-implementations_amd"))
import torch  # noqa: F401,E402  (one HIP runtime: torch first)
import zk_amd  # noqa: E402
from zk_amd.gkr import Circuit, Operation, prove  # noqa: E402

log_inputs = int(sys.argv[1]) if len(sys.argv) > 1 else 12
rng = random.Random(11)
structure = [[rng.choice((Operation.Add, Operation.Mul)) for _ in range(1 << (log_inputs - 1 - i))]
             for i in range(log_inputs)]
p = zk_amd.modulus(0)
inputs = [rng.randrange(p) for _ in range(1 << log_inputs)]
circ = Circuit(structure, 0)
ctx = zk_amd.Context(0)
for i in range(3):
    print(f"--- prove {i}", file=sys.stderr, flush=True)
    prove(circ, inputs, ctx)
ctx.close()
