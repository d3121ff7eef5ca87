"""ctypes binding of libzksumcheck.so (include/zk_sumcheck.h).

The library is the product: HIP kernels for gfx950 plus the C++ host
orchestration. Loading it never falls back to anything else — if the shared
object is missing this module raises, and creating a context on a machine
without a gfx950 GPU fails with ZK_EDEVICE.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ZK_LIB_PATH") or os.path.join(_HERE, "_lib", "libzksumcheck.so")  # override: A/B builds
PKG_ROOT = os.path.dirname(_HERE)

ZK_OK, ZK_EINVAL, ZK_EDEVICE, ZK_ECOMM, ZK_ENOMEM, ZK_EUNSUPPORTED = range(6)
ZK_BLOB_GKR, ZK_BLOB_SUMCHECK = 1, 2
ERROR_NAMES = {1: "ZK_EINVAL", 2: "ZK_EDEVICE", 3: "ZK_ECOMM", 4: "ZK_ENOMEM", 5: "ZK_EUNSUPPORTED"}
ABI_VERSION = 15  # ZK_ABI_VERSION in include/zk_sumcheck.h: the ZkStats layout and the signatures below
KERNEL_KINDS = ["gkr_round0", "gkr_round", "sc_round", "fold", "reduce", "convert", "synth", "layer", "msm", "gkr_round_lanes", "gkr_tail", "gkr_dround", "gkr_dtail", "gkr_d0", "gkr_dm", "gkr_t33", "coll"]


class ZkError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


class ZkStats(C.Structure):
    _fields_ = [
        ("launches", C.c_uint64 * len(KERNEL_KINDS)),
        ("kernel_ms", C.c_double * len(KERNEL_KINDS)),
        ("alg_bytes", C.c_double * len(KERNEL_KINDS)),
        ("field_muls", C.c_double * len(KERNEL_KINDS)),
        ("host_syncs", C.c_uint64),
        ("collectives", C.c_uint64),
        ("host_wait_us", C.c_double),
        ("host_work_us", C.c_double),
        ("device_fs_rounds", C.c_uint64),
    ]


class ZkLaunch(C.Structure):
    _fields_ = [("kind", C.c_int), ("ms", C.c_double), ("alg_bytes", C.c_double)]


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t)

# name -> (restype, argtypes); every symbol declared in include/zk_sumcheck.h
P, I, U32, U64, SZ = C.c_void_p, C.c_int, C.c_uint32, C.c_uint64, C.c_size_t
SIGNATURES = {
    "zk_abi_version": (U32, []),
    "zk_last_error": (C.c_char_p, []),
    "zk_ctx_create": (I, [I, C.POINTER(C.c_void_p)]),
    "zk_ctx_destroy": (None, [P]),
    "zk_ctx_set_timing": (I, [P, I]),
    "zk_ctx_set_timing_mask": (I, [P, U32]),
    "zk_ctx_get_stats": (I, [P, C.POINTER(ZkStats)]),
    "zk_ctx_reset_stats": (I, [P]),
    "zk_ctx_get_launches": (I, [P, P, SZ, C.POINTER(SZ)]),
    "zk_transcript_new": (P, []),
    "zk_transcript_clone": (P, [P]),
    "zk_transcript_free": (None, [P]),
    "zk_transcript_append": (I, [P, P, SZ]),
    "zk_transcript_get_random_challenge": (I, [P, I, I, P]),
    "zk_transcript_serialize": (I, [P, P, SZ, C.POINTER(SZ)]),
    "zk_transcript_deserialize": (P, [P, SZ]),
    "zk_fe_vec_to_bytes": (I, [I, I, P, SZ, P]),
    "zk_mle_partial_evaluate": (I, [P, I, I, P, U32, U32, P, P]),
    "zk_mle_evaluate": (I, [P, I, I, P, U32, P, U32, P]),
    "zk_mle_binop": (I, [P, I, I, I, P, U32, P, U32, P]),
    "zk_mle_scale": (I, [P, I, I, P, U32, P, P]),
    "zk_mle_tensor": (I, [P, I, I, I, P, U64, P, U64, P]),
    "zk_sumcheck_prove": (I, [P, I, I, P, U32, P, P]),
    "zk_sumcheck_verify": (I, [P, I, I, P, U32, P, U32, U32, P, C.POINTER(C.c_int)]),
    "zk_gkr_sumcheck_prove": (I, [P, I, I, P, U32, P, P, P, P, P, P]),
    "zk_gkr_sumcheck_verify": (I, [I, I, P, P, U32, P, P, C.POINTER(C.c_int), P, P]),
    "zk_gkr_circuit_rounds": (I, [U32, P, C.POINTER(U32)]),
    "zk_gkr_circuit_prove": (I, [P, I, I, U32, P, P, P, U32, P, P, P, P, P, P]),
    "zk_gkr_circuit_verify": (I, [I, I, U32, P, P, P, U32, P, P, P, P, P, C.POINTER(C.c_int)]),
    "zk_gkr_circuit_prove_kzg": (I, [P, I, U32, P, P, P, U32, P, P, P, P, P, P, P, P, P, P]),
    "zk_gkr_circuit_verify_kzg": (I, [I, U32, P, P, P, P, P, P, P, P, P, P, C.POINTER(C.c_int)]),
    "zk_kzg_setup": (I, [P, I, P, U32, C.POINTER(C.c_void_p)]),
    "zk_kzg_free": (None, [P]),
    "zk_kzg_lagrange_basis": (I, [P, P, U32, P]),
    "zk_kzg_commit": (I, [P, P, I, P, P]),
    "zk_dev_kzg_commit": (I, [P, P, P, P]),
    "zk_kzg_get_proof": (I, [P, P, I, P, P, P, P]),
    "zk_dev_kzg_get_proof": (I, [P, P, I, P, P, P, P]),
    "zk_kzg_release_fixed_base_cache": (I, [I]),
    "zk_msm_g1": (I, [P, I, P, P, SZ, P]),
    "zk_kzg_g2_taus": (I, [P, P]),
    "zk_kzg_verify": (I, [I, P, P, P, U32, P, U32, P, C.POINTER(C.c_int)]),
    "zk_g2_mul_generator": (I, [I, P, SZ, P]),
    "zk_bls12_381_pairing": (I, [P, P, P]),
    "zk_bls12_381_pairing_check": (I, [P, P, SZ, C.POINTER(C.c_int)]),
    "zk_gkr_proof_to_blob": (I, [I, I, P, P, U32, P, P, SZ, C.POINTER(SZ)]),
    "zk_sumcheck_proof_to_blob": (I, [I, I, P, U32, U32, P, P, SZ, C.POINTER(SZ)]),
    "zk_proof_blob_info": (I, [P, SZ, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(U32)]),
    "zk_gkr_proof_from_blob": (I, [P, SZ, I, P, P, U32, P]),
    "zk_sumcheck_proof_from_blob": (I, [P, SZ, I, P, SZ, C.POINTER(U32), P]),
    "zk_gkr_verify_blob": (I, [P, SZ, P, C.POINTER(C.c_int), P, P, U32]),
    "zk_keccak256": (I, [P, SZ, P]),
    "zk_dev_alloc": (I, [P, SZ, C.POINTER(C.c_void_p)]),
    "zk_dev_free": (I, [P, P]),
    "zk_dev_upload": (I, [P, I, I, P, SZ, P]),
    "zk_dev_download": (I, [P, I, I, P, SZ, P]),
    "zk_dev_synth_fill": (I, [P, I, P, U64, U64, U32, U64, U64]),
    "zk_dev_mle_partial_evaluate": (I, [P, I, P, U32, U32, I, P, P]),
    "zk_dev_mle_tensor": (I, [P, I, I, P, U64, P, U64, P]),
    "zk_dev_gkr_sumcheck_prove": (I, [P, I, P, U32, I, P, P, P, P, P]),
    "zk_ctx_attach_host_comm": (I, [P, I, I, ALLREDUCE_FN, P]),
    "zk_comm_get_unique_id": (I, [P]),
    "zk_ctx_attach_rccl": (I, [P, I, I, P]),
    "zk_ctx_detach_comm": (I, [P]),
    "zk_ctx_comm_count": (I, [P, C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "zk_ctx_attach_peer_reduce": (I, [P, I, C.POINTER(I)]),
    "zk_dev_gkr_sumcheck_prove_sharded": (I, [P, I, P, U32, I, P, P, P, P, P]),
}

_lib = None


def lib():
    """Load the HIP library (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make -C {PKG_ROOT}` "
                "(or __graft_entry__.build()); the prover has no CPU fallback"
            )
        # One HIP runtime per process: torch's libtorch_hip NEEDs the unversioned
        # libamdhip64.so / librccl.so from its own lib dir, which the loader does not
        # match against an already-loaded /opt/rocm libamdhip64.so.7, so loading us
        # first and torch later leaves two runtimes that double-free at exit. Load
        # torch's copies first; our NEEDED sonames (libamdhip64.so.7, librccl.so.1)
        # then bind to them.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        L.zk_abi_version.restype = C.c_uint32
        L.zk_abi_version.argtypes = []
        got = L.zk_abi_version()
        if got != ABI_VERSION:
            raise ImportError(
                f"{LIB_PATH} has ABI version {got}, this binding expects {ABI_VERSION} "
                f"(stale build?): rebuild it with `make -C {PKG_ROOT}`"
            )
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(code: int) -> None:
    if code != ZK_OK:
        raise ZkError(code, lib().zk_last_error().decode(errors="replace"))
