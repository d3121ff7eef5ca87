import os, sys, ctypes as C
sys.path.insert(0, "zk-research-implementations_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np
import zk_amd
from zk_amd._lib import check, lib
from zk_amd.elems import as_limbs, ptr, to_ints
import coracle as co
def prove(ctx, field, n):
    tabs = [ctx.synth(field, 1 << n, seed=23, table=t) for t in range(4)]
    arr = (C.c_void_p * 4)(*[t.ptr.value for t in tabs])
    coeffs = np.zeros((n, 3, 4), np.uint64); nco = np.zeros(n, np.uint8); ch = np.zeros((n, 4), np.uint64)
    tr = zk_amd.Transcript(field)
    check(lib().zk_dev_gkr_sumcheck_prove_sharded(ctx.h, field, arr, n, 0, ptr(as_limbs([0])), tr.h, ptr(coeffs), ptr(nco), ptr(ch)))
    return [to_ints(coeffs[k, : nco[k]]) for k in range(n)], to_ints(ch)
for pre in ("0", "1"):
    os.environ["ZK_PRELAUNCH"] = pre
    for n in (11, 12, 13, 14, 16, 17, 20):
        tabs = [co.synth(0, 23, t, 0, 1 << n) for t in range(4)]
        polys, chal = co.gkr_prove(0, tabs, co.Transcript())
        want = ([list(p) for p in polys], list(chal))
        ctx = zk_amd.Context(0)
        try:
            got = prove(ctx, 0, n)
            bad = [k for k in range(n) if got[0][k] != want[0][k]]
            print("pre", pre, "n", n, "OK" if got == want else f"MISMATCH first bad round {bad[:3]}", flush=True)
        except Exception as e:
            print("pre", pre, "n", n, "ERR", e, flush=True)
        finally:
            ctx.close()
