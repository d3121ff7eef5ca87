"""Several independent 24-variable GKR proofs in flight on ONE MI355X: K host
threads, each with its own context (stream, pinned page, workspaces) proving
over the same device-resident tables (read only) with fresh transcripts —
the serving shape (many proofs, one GPU). Reports the aggregate proofs/s and
the per-proof latency for K = 1 .. KMAX, and checks every proof's challenges
against the K = 1 proof. usage: python tools/serve_streams.py [KMAX] [PROOFS_PER_THREAD]"""
import ctypes as C
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zk-research-implementations_amd"))
import zk_amd  # noqa: E402
from zk_amd._lib import check, lib  # noqa: E402
from zk_amd.elems import as_limbs, ptr  # noqa: E402

NV, FIELD, SEED = 24, 0, 3
kmax = int(sys.argv[1]) if len(sys.argv) > 1 else 3
per = int(sys.argv[2]) if len(sys.argv) > 2 else 40

owner = zk_amd.Context(0)
tabs = [owner.synth(FIELD, 1 << NV, seed=SEED, table=t) for t in range(4)]
arr = (C.c_void_p * 4)(*[t.ptr.value for t in tabs])
zero = as_limbs([0])


def prove(ctx, out_ch):
    coeffs = np.zeros((NV, 3, 4), np.uint64)
    nco = np.zeros(NV, np.uint8)
    tr = zk_amd.Transcript(FIELD)
    check(lib().zk_dev_gkr_sumcheck_prove_sharded(ctx.h, FIELD, arr, NV, 0, ptr(zero), tr.h, ptr(coeffs), ptr(nco),
                                                  ptr(out_ch)))


ref = np.zeros((NV, 4), np.uint64)
prove(owner, ref)
for k in range(1, kmax + 1):
    ctxs = [zk_amd.Context(0) for _ in range(k)]
    lat = [[] for _ in range(k)]
    ok = [True] * k
    for c in ctxs:  # warm-up (workspaces, code objects)
        ch = np.zeros((NV, 4), np.uint64)
        for _ in range(3):
            prove(c, ch)
    barrier = threading.Barrier(k + 1)

    def run(i):
        ch = np.zeros((NV, 4), np.uint64)
        barrier.wait()
        for _ in range(per):
            t0 = time.perf_counter()
            prove(ctxs[i], ch)
            lat[i].append(time.perf_counter() - t0)
            ok[i] = ok[i] and np.array_equal(ch, ref)

    th = [threading.Thread(target=run, args=(i,)) for i in range(k)]
    for t in th:
        t.start()
    barrier.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    alll = sorted(x for l in lat for x in l)
    print(f"K={k}: {k * per} proofs in {wall * 1e3:.1f} ms -> {k * per / wall:.0f} proofs/s "
          f"({wall * 1e3 / (k * per):.4f} ms per proof aggregate; {32 * ((1 << NV) - 1) * k * per / wall / 1e9:.1f} G field-ops/s), "
          f"latency median {alll[len(alll) // 2] * 1e3:.3f} ms p90 {alll[int(len(alll) * 0.9)] * 1e3:.3f} ms, "
          f"all proofs equal: {all(ok)}", flush=True)
    for c in ctxs:
        c.close()
