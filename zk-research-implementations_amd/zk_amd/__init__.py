"""zk_amd — MI355X-native sum-check / GKR sum-check prover.

Python mirror of the reference crates' API (obah/zk-research-implementations):
  fiat_shamir::fiat_shamir_transcript::{Transcript, fq_vec_to_bytes}
  multilinear_polynomial::{MultilinearPoly, ProductPoly, SumPoly}
  univariate_polynomial::UnivariatePoly
  sum_check::sum_check_protocol::{prove, verify, gkr_prove, gkr_verify, Proof, GkrProof, GkrVerify}
over the C ABI of include/zk_sumcheck.h. Every table-sized operation runs in
the HIP library on a gfx950 GPU; this module only marshals arguments.

Field elements are canonical Python ints, or numpy uint64 arrays of shape
[n, 4] (little-endian limbs) for tables.
"""
from __future__ import annotations

from .api import (  # noqa: F401
    Field,
    GkrProof,
    GkrVerify,
    MultilinearPoly,
    ProductPoly,
    Proof,
    SumPoly,
    Transcript,
    UnivariatePoly,
    blob_info,
    default_context,
    fq_vec_to_bytes,
    gkr_prove,
    gkr_verify,
    gkr_verify_blob,
    keccak256,
    modulus,
    prove,
    verify,
)
from .context import Context, DeviceTable  # noqa: F401
from . import gkr  # noqa: F401  (gkr crate mirror: Circuit, Operation, prove, verify)
from ._lib import ZkError  # noqa: F401
