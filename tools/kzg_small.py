"""Repeated small KZG commits (latency of a small MSM); usage: python tools/kzg_small.py NV REPS"""
import os
import random
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zk-research-implementations_amd"))
import zk_amd  # noqa: E402
from zk_amd.kzg import KZG  # noqa: E402

nv, reps = int(sys.argv[1]), int(sys.argv[2])
ctx = zk_amd.Context(0)
p = zk_amd.modulus(2)
rng = random.Random(nv)
k = KZG([rng.randrange(p) for _ in range(nv)], ctx)
ev = [rng.randrange(p) for _ in range(1 << nv)]
k.commit(ev)
t0 = time.perf_counter()
for _ in range(reps):
    k.commit(ev)
print(f"nv {nv}: {1e3 * (time.perf_counter() - t0) / reps:.3f} ms per commit")
