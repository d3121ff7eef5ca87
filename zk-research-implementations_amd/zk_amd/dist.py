"""Multi-GPU plumbing: one process per GPU, torch.distributed for rendezvous.

The hypercube of a GKR sum-check over n = n_local + log2(world) variables is
split by its LOW index bits: rank g holds global indices m * world + g, so the
fold pair (j, j + N/2) of every round stays local for the first n_local rounds
(zk_sumcheck.h, "Multi-GPU"). Partial round sums cross ranks as limb-split
u64 vectors (each 256-bit element as eight 32-bit limbs in u64 lanes), whose
plain integer SUM is exact; the receiver folds the limbs back mod p.

Data path: RCCL (`Context.attach_rccl`, ncclAllReduce on the ctx stream over
xGMI). `TorchAllreduce` is the host-memory alternative over any
torch.distributed backend (gloo on CPU, or to share one GPU between ranks in
tests, which RCCL refuses).
"""
from __future__ import annotations

import numpy as np


def shard_layout(rank: int, world: int) -> tuple[int, int]:
    """(index0, stride) of this rank's shard: local m <-> global m * world + rank."""
    if world & (world - 1) or not 0 <= rank < world:
        raise ValueError("world must be a power of two and 0 <= rank < world")
    return rank, world


def limb_split(values) -> np.ndarray:
    """Field elements (ints < 2^256) -> u64[8 * len] of 32-bit limbs."""
    out = np.zeros(8 * len(values), dtype=np.uint64)
    for k, v in enumerate(values):
        v = int(v)
        for i in range(8):
            out[8 * k + i] = (v >> (32 * i)) & 0xFFFFFFFF
    return out


def limb_join(words: np.ndarray, p: int) -> list[int]:
    """Inverse of limb_split after a SUM over ranks: each element mod p."""
    w = np.asarray(words, dtype=np.uint64).reshape(-1, 8)
    return [sum(int(x) << (32 * i) for i, x in enumerate(row)) % p for row in w]


class TorchAllreduce:
    """In-place u64 SUM over a torch.distributed group (host memory)."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        self._torch, self._dist, self.group = torch, dist, group

    def __call__(self, arr: np.ndarray) -> None:
        t = self._torch.from_numpy(arr.view(np.int64))  # shares memory; values < 2^63
        self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM, group=self.group)


def rendezvous_rccl(ctx, rank: int, world: int) -> None:
    """Rank 0 creates the RCCL unique id; torch.distributed broadcasts it."""
    import torch.distributed as dist

    from .context import rccl_unique_id

    obj = [rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    ctx.attach_rccl(rank, world, obj[0])
