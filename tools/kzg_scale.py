"""KZG setup / commit timings at growing sizes (BLS12-381 G1) on one GPU.
usage: python tools/kzg_scale.py 16 20 24"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-research-implementations_amd"))
import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402

import zk_amd  # noqa: E402
from zk_amd._lib import check, lib  # noqa: E402
from zk_amd.kzg import KZG  # noqa: E402

ctx = zk_amd.default_context()
R = zk_amd.modulus(2)
for nv in map(int, sys.argv[1:]):
    rng = random.Random(nv)
    taus = [rng.randrange(R) for _ in range(nv)]
    t0 = time.perf_counter()
    k = KZG(taus, ctx)
    t_setup = time.perf_counter() - t0
    dev = ctx.synth(2, 1 << nv, seed=5, table=0)
    out = np.zeros((1, 12), np.uint64)
    check(lib().zk_dev_kzg_commit(ctx.h, k.h, dev.ptr, out.ctypes.data_as(C.c_void_p)))  # warm-up
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        check(lib().zk_dev_kzg_commit(ctx.h, k.h, dev.ptr, out.ctypes.data_as(C.c_void_p)))
        ts.append(time.perf_counter() - t0)
    t_commit = sorted(ts)[1]
    print(f"nv {nv}: setup {t_setup * 1e3:.1f} ms, commit (2^{nv}-point MSM) {t_commit * 1e3:.2f} ms, "
          f"{(1 << nv) / t_commit / 1e6:.1f} M points/s, commitment x lo {int(out[0][0]):016x}", flush=True)
    k.close()
    del dev
