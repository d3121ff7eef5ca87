"""One rank of a sharded GKR sum-check on the GPU (spawned by
tests/test_gpu_sharded.py; not a test module itself).

env: RANK, WORLD_SIZE, MASTER_PORT, COMM in {host, rccl, none}, FIELD, NLOCAL, OUT
(+ optional SEED, default 19; PEER=1: zk_ctx_attach_peer_reduce after the
communicator, so the steps' sums meet in the ranks' IPC-mapped buffers;
PEER_MAY_FAIL=1: a refused attach is recorded, and the proof runs on the
communicator)
Rank g proves its low-index-bit shard; rank 0 writes the proof as JSON.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zk-research-implementations_amd"))


def main() -> None:
    import numpy as np
    import torch.distributed as dist

    import zk_amd
    from zk_amd._lib import check, lib
    from zk_amd.dist import TorchAllreduce, rendezvous_rccl, shard_layout
    from zk_amd.elems import as_limbs, ptr, to_ints

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    comm, field, nloc = os.environ["COMM"], int(os.environ["FIELD"]), int(os.environ["NLOCAL"])
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{os.environ['MASTER_PORT']}", rank=rank,
                            world_size=world)
    ctx = zk_amd.Context(0)
    if comm == "host":
        ctx.attach_host_comm(rank, world, TorchAllreduce())
    elif comm == "rccl":
        rendezvous_rccl(ctx, rank, world)
    peer_refused = None
    if os.environ.get("PEER") == "1":
        try:
            ctx.attach_peer_reduce()
        except zk_amd.ZkError as e:  # (PEER_MAY_FAIL=1: the test checks every rank refused)
            if os.environ.get("PEER_MAY_FAIL") != "1":
                raise
            peer_refused = str(e)
        ctx.reset_stats()  # (the handle exchange went through the communicator)
    i0, stride = shard_layout(rank, world)
    seed = int(os.environ.get("SEED", "19"))
    tabs = [ctx.synth(field, 1 << nloc, seed=seed, table=t, index0=i0, stride=stride) for t in range(4)]
    n = nloc + world.bit_length() - 1
    arr = (C.c_void_p * 4)(*[t.ptr.value for t in tabs])
    coeffs = np.zeros((max(n, 1), 3, 4), np.uint64)
    nco = np.zeros(max(n, 1), np.uint8)
    ch = np.zeros((max(n, 1), 4), np.uint64)
    tr = zk_amd.Transcript(field)
    check(lib().zk_dev_gkr_sumcheck_prove_sharded(ctx.h, field, arr, nloc, 0, ptr(as_limbs([0])), tr.h, ptr(coeffs),
                                                  ptr(nco), ptr(ch)))
    polys = [to_ints(coeffs[k, : nco[k]]) for k in range(n)]
    for t in tabs:
        t.free()
    blob = zk_amd.GkrProof([zk_amd.UnivariatePoly(p, field) for p in polys], 0, []).to_bytes(field)
    c = (polys[0] + [0, 0, 0])[:3] if n else [0, 0, 0]
    claimed = (2 * c[0] + c[1] + c[2]) % zk_amd.modulus(field)  # s_0(0) + s_0(1), as the fixtures hold it
    blob_c = zk_amd.GkrProof([zk_amd.UnivariatePoly(p, field) for p in polys], claimed, []).to_bytes(field)
    res = {"polys": [[hex(x) for x in p] for p in polys],
           "chal": [hex(x) for x in to_ints(ch[:n])], "collectives": ctx.stats()["collectives"],
           "blob_keccak": zk_amd.keccak256(blob).hex(), "blob_keccak_claimed": zk_amd.keccak256(blob_c).hex(),
           "comm": ctx.comm_info(), "peer": ctx.peer_reduce, "peer_refused": peer_refused}
    with open(os.path.join(os.environ["OUT"], f"rank{rank}.json"), "w") as fh:
        json.dump(res, fh)
    dist.barrier()
    dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
