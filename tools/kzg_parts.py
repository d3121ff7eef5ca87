import os, sys, time, random
sys.path.insert(0, "zk-research-implementations_amd")
import zk_amd
from zk_amd.kzg import KZG
from zk_amd.gkr import Circuit, Operation, prove
from zk_amd.elems import as_limbs
ctx = zk_amd.Context(0)
p = zk_amd.modulus(2)
rng = random.Random(14)
for nv in (10, 14, 16):
    taus = [rng.randrange(p) for _ in range(nv)]
    ev = [rng.randrange(p) for _ in range(1 << nv)]
    for rep in range(2):
        t0 = time.perf_counter(); k = KZG(taus, ctx); t1 = time.perf_counter()
        c = k.commit(ev); t2 = time.perf_counter()
        pt = [rng.randrange(p) for _ in range(nv)]
        v = k.open(pt, ev); t3 = time.perf_counter()
        pr = k.get_proof(v, pt, ev); t4 = time.perf_counter()
        g2 = k.g2_taus; t5 = time.perf_counter()
        print(f"nv {nv}: setup {1e3*(t1-t0):.1f} commit {1e3*(t2-t1):.1f} open {1e3*(t3-t2):.1f} get_proof {1e3*(t4-t3):.1f} g2 {1e3*(t5-t4):.1f} ms", flush=True)
        k.close()
structure = [[rng.choice((Operation.Add, Operation.Mul)) for _ in range(1 << (13 - i))] for i in range(14)]
circ = Circuit(structure, 2)
x = as_limbs([rng.randrange(p) for _ in range(1 << 14)])
taus = [rng.randrange(p) for _ in range(14)]
for rep in range(3):
    t0 = time.perf_counter(); prove(circ, x, ctx); t1 = time.perf_counter(); prove(circ, x, ctx, taus=taus); t2 = time.perf_counter()
    print(f"circuit 2^14: plain {1e3*(t1-t0):.1f} ms, with KZG {1e3*(t2-t1):.1f} ms", flush=True)
