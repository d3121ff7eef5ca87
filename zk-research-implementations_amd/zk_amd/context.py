"""Device context and device-resident tables (zk_ctx / zk_dev_* of the C ABI)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import KERNEL_KINDS, check, lib
from .elems import as_limbs, ptr, to_ints

REPR_CANONICAL, REPR_MONTGOMERY = 0, 1


class Context:
    """One HIP device + stream + workspace (+ optional communicator)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib().zk_ctx_create(int(device), C.byref(h)))
        self.h = h
        self.device = device
        self._callbacks = None  # keep ctypes callbacks alive while attached
        self.peer_reduce = False  # zk_ctx_attach_peer_reduce succeeded

    def close(self) -> None:
        if getattr(self, "h", None):
            lib().zk_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- stats ----
    def set_timing(self, enable: bool) -> None:
        check(lib().zk_ctx_set_timing(self.h, int(bool(enable))))

    def set_timing_kinds(self, kinds) -> None:
        """Time only launches of these kernel kinds (names from KERNEL_KINDS)."""
        mask = 0
        for k in kinds:
            mask |= 1 << KERNEL_KINDS.index(k)
        check(lib().zk_ctx_set_timing_mask(self.h, mask))

    def reset_stats(self) -> None:
        check(lib().zk_ctx_reset_stats(self.h))

    def stats(self) -> dict:
        s = _lib.ZkStats()
        check(lib().zk_ctx_get_stats(self.h, C.byref(s)))
        return {
            "kernels": {
                k: {
                    "launches": int(s.launches[i]),
                    "ms": float(s.kernel_ms[i]),
                    "alg_bytes": float(s.alg_bytes[i]),
                    "field_muls": float(s.field_muls[i]),
                }
                for i, k in enumerate(KERNEL_KINDS)
            },
            "host_syncs": int(s.host_syncs),
            "collectives": int(s.collectives),
            "host_wait_us": float(s.host_wait_us),
            "device_fs_rounds": int(s.device_fs_rounds),
            "host_work_us": float(s.host_work_us),
        }

    def launches(self) -> list:
        """Event-timed launches since the last reset_stats, in order: (kind, ms, alg_bytes)."""
        n = C.c_size_t(0)
        check(lib().zk_ctx_get_launches(self.h, None, 0, C.byref(n)))
        arr = (_lib.ZkLaunch * max(1, n.value))()
        check(lib().zk_ctx_get_launches(self.h, arr, n.value, C.byref(n)))
        return [{"kind": KERNEL_KINDS[a.kind], "ms": a.ms, "alg_bytes": a.alg_bytes} for a in arr[: n.value]]

    # ---- device tables ----
    def alloc(self, field: int, count: int) -> "DeviceTable":
        return DeviceTable(self, field, count)

    def upload(self, field: int, values, repr: int = REPR_CANONICAL) -> "DeviceTable":
        a = as_limbs(values)
        t = DeviceTable(self, field, a.shape[0])
        check(lib().zk_dev_upload(self.h, field, repr, ptr(a), a.shape[0], t.ptr))
        return t

    def synth(self, field: int, count: int, seed: int, table: int, index0: int = 0, stride: int = 1) -> "DeviceTable":
        t = DeviceTable(self, field, count)
        check(lib().zk_dev_synth_fill(self.h, field, t.ptr, count, seed, table, index0, stride))
        return t

    # ---- communicators ----
    def attach_rccl(self, rank: int, world: int, unique_id: bytes) -> None:
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(unique_id))
        self.peer_reduce = False  # (a new communicator releases the peer buffers)
        check(lib().zk_ctx_attach_rccl(self.h, rank, world, buf))

    def attach_host_comm(self, rank: int, world: int, allreduce) -> None:
        """allreduce(np.ndarray[uint64]) -> None: in-place SUM over all ranks."""

        def _ar(user, data, count):
            try:
                allreduce(np.ctypeslib.as_array(data, shape=(count,)))
                return 0
            except Exception:  # the C side turns this into ZK_ECOMM
                return 1

        cb = _lib.ALLREDUCE_FN(_ar)
        self.peer_reduce = False
        check(lib().zk_ctx_attach_host_comm(self.h, rank, world, cb, None))
        self._callbacks = cb

    def detach_comm(self) -> None:
        check(lib().zk_ctx_detach_comm(self.h))
        self._callbacks = None
        self.peer_reduce = False

    def attach_peer_reduce(self, enable: bool = True) -> None:
        """Collective (every rank, after attaching a communicator, world <= 8):
        the sharded steps' sums meet in the ranks' IPC-mapped receive buffers,
        summed by the step kernels themselves, instead of an all-reduce on the
        communicator (which still carries the gather). Checked once across
        the world on attach; raises ZkError if a buffer cannot be opened or the
        check fails (the context then keeps the communicator's all-reduce)."""
        ok = C.c_int(0)
        self.peer_reduce = False
        check(lib().zk_ctx_attach_peer_reduce(self.h, 1 if enable else 0, C.byref(ok)))
        self.peer_reduce = bool(ok.value)

    def comm_info(self) -> dict:
        """{"kind": "none"|"host"|"rccl", "rank": r, "count": n}; for RCCL the
        rank and count are what the communicator reports (ncclCommUserRank /
        ncclCommCount)."""
        kind, rank, count = C.c_int(), C.c_int(), C.c_int()
        check(lib().zk_ctx_comm_count(self.h, C.byref(kind), C.byref(rank), C.byref(count)))
        return {"kind": ("none", "host", "rccl")[kind.value], "rank": rank.value, "count": count.value}


def rccl_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    check(lib().zk_comm_get_unique_id(buf))
    return bytes(buf)


class DeviceTable:
    """A device buffer of `count` Montgomery field elements (32 B each)."""

    def __init__(self, ctx: Context, field: int, count: int):
        self.ctx, self.field, self.count = ctx, field, int(count)
        p = C.c_void_p()
        check(lib().zk_dev_alloc(ctx.h, max(1, self.count) * 32, C.byref(p)))
        self.ptr = p

    def free(self) -> None:
        if getattr(self, "ptr", None) and self.ctx.h:
            lib().zk_dev_free(self.ctx.h, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def download(self, repr: int = REPR_CANONICAL) -> np.ndarray:
        out = np.zeros((self.count, 4), np.uint64)
        check(lib().zk_dev_download(self.ctx.h, self.field, repr, self.ptr, self.count, ptr(out)))
        return out

    def to_ints(self) -> list[int]:
        return to_ints(self.download())
