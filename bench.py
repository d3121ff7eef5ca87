"""Benchmark: GKR sum-check prover (BASELINE.json metric) on MI355X.

One step = one full `gkr_prove` (sum_check_protocol.rs:86-115) over the
composed polynomial A*S + M*P whose four tables are already resident in HBM
(BASELINE config 3: 24 variables per GPU, BN254 Fr, synthetic uniform tables,
seed 3). With --gpus N (torchrun, one process per GPU) the hypercube has
24 + log2(N) variables, rank g holding the sub-cube whose low log2(N) index bits
equal g; each round does one RCCL all-reduce of the partial sums (weak scaling:
per-GPU table size fixed).

value = canonical field ops / s of the whole job = 32 * (2^n - 1) * steps / time
(SURVEY.md 8(d)); ms_per_step = prover milliseconds per proof.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zk-research-implementations_amd"))

FIELDS = {"bn254_fr": 0, "bn254_fq": 1, "bls12_381_fr": 2}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # a proof takes ~1.1 ms: 100 timed proofs after 20 warm-up ones are the
    # steady state (10 after 3 read ~4 % slower: clocks still ramping)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--nvars", type=int, default=24, help="variables per GPU")
    ap.add_argument("--field", default="bn254_fr", choices=sorted(FIELDS))
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--cpu-sample-nvars", type=int, default=24,
                    help="size of the single-thread reference-faithful CPU run (24 = the headline workload)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fold", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-tables (PCIe-inclusive) prove")
    ap.add_argument("--no-serving", action="store_true", help="skip the two-proofs-in-flight serving leg")
    ap.add_argument("--cpu-fast-nvars", type=int, default=24, help="size of the OpenMP CPU restatement run")
    ap.add_argument("--no-circuit", action="store_true", help="skip the full GKR circuit prove (SURVEY 8(f2))")
    ap.add_argument("--no-config5", action="store_true", help="skip BLS12-381 GKR + KZG commit (BASELINE config 5)")
    ap.add_argument("--no-config4", dest="config4", action="store_false",
                    help="skip the 26-variable-total proof split over all ranks (BASELINE config 4, strong scaling)")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                    help="N>1 data path: RCCL (default) or, as a diagnostic that rehearses the multi-rank bench "
                    "on one card, a gloo host all-reduce with every rank on device LOCAL_RANK %% device_count")
    ap.add_argument("--force-rccl", action="store_true",
                    help="diagnostic: at world 1 route every step through ncclAllReduce (the multi-rank data path)")
    ap.add_argument("--reduce", default="comm", choices=["comm", "peer"],
                    help="N>1 (or --force-rccl): each step's sums through an all-reduce on the communicator (default) "
                    "or through the ranks' IPC-mapped peer buffers, summed by the step kernels (zk_ctx_attach_peer_reduce)")
    ap.add_argument("--no-peer-leg", action="store_true",
                    help="N>1: skip the side leg that reruns the headline with --reduce peer in fresh ranks")
    ap.add_argument("--no-events", action="store_true", help="diagnostic: time without per-launch HIP events")
    ap.add_argument("--no-plain", action="store_true",
                    help="skip BASELINE config 1 (12-var plain prove, CPU port) and the GPU plain prove/verify legs")
    return ap.parse_args()


def golden_key(field: int, n: int, seed: int) -> str:
    return f"{[k for k, v in FIELDS.items() if v == field][0]}_{n}_s{seed}"


def proof_check(field: int, n: int, seed: int, coeffs, nco, ch) -> dict:
    """Keccak-256 of the proof blob (claimed sum = s_0(0) + s_0(1)), written
    by the library's serialiser (zk_gkr_proof_to_blob), against the committed
    full-size oracle fixture for this workload (tests/golden/large.json, from
    oracle/zk_oracle.c or_gkr_prove_fast via tests/golden/make_large_golden.py)
    when one exists. A mismatch aborts the bench: a wrong proof has no rate."""
    from zk_amd.elems import to_ints

    return proof_digest_check(field, n, seed, [to_ints(coeffs[k, : nco[k]]) for k in range(n)], to_ints(ch))


def proof_digest_check(field: int, n: int, seed: int, polys, chal, abort: bool = True) -> dict:
    """proof_check on a proof given as Python ints (trimmed coefficient lists
    per round, challenges)."""
    import zk_amd

    p = zk_amd.modulus(field)
    c = polys[0] + [0] * (3 - len(polys[0]))
    claimed = (2 * c[0] + c[1] + c[2]) % p
    blob = zk_amd.GkrProof([zk_amd.UnivariatePoly(q, field) for q in polys], claimed, chal).to_bytes(field)
    dig = zk_amd.keccak256(blob).hex()
    key = golden_key(field, n, seed)
    path = os.path.join(ROOT, "tests", "golden", "large.json")
    fix = json.load(open(path)).get(key) if os.path.exists(path) else None
    out = {"blob_keccak256": dig, "fixture": f"tests/golden/large.json[{key}]" if fix else None,
           "matches_oracle_fixture": (dig == fix["blob_keccak256"]) if fix else None}
    if abort and fix and dig != fix["blob_keccak256"]:
        raise SystemExit(f"proof digest {dig} != oracle fixture {fix['blob_keccak256']} ({key})")
    return out


def kzg_commit_check(nvars: int, out) -> dict:
    """The config-5 commitment (affine x, y limbs) against the committed fixture
    f(taus) * G1 (tests/golden/kzg.json, from the C oracle's MLE evaluation and
    kzg_oracle.mul via tests/golden/make_kzg_golden.py). A mismatch aborts the
    bench, as for the proof digest."""
    x = sum(int(out[0, i]) << (64 * i) for i in range(6))
    y = sum(int(out[0, 6 + i]) << (64 * i) for i in range(6))
    key = f"bls12_381_fr_{nvars}_s5"
    path = os.path.join(ROOT, "tests", "golden", "kzg.json")
    fix = json.load(open(path)).get(key) if os.path.exists(path) else None
    if fix and (x, y) != (int(fix["commit_x"], 16), int(fix["commit_y"], 16)):
        raise SystemExit(f"KZG commitment ({x:#x}, {y:#x}) != oracle fixture ({key})")
    return {"fixture": f"tests/golden/kzg.json[{key}]" if fix else None, "matches_oracle_fixture": bool(fix) or None}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def _ranges(cpus) -> str:
    """[0,1,2,5] -> '0-2,5'"""
    out, start, prev = [], None, None
    for c in cpus:
        if start is None:
            start = prev = c
        elif c == prev + 1:
            prev = c
        else:
            out.append(f"{start}-{prev}" if prev > start else f"{start}")
            start = prev = c
    if start is not None:
        out.append(f"{start}-{prev}" if prev > start else f"{start}")
    return ",".join(out)


def config1_bench(ctx, field: int, nvars: int = 12, runs: int = 101) -> dict:
    """BASELINE config 1: the reference's own benchmark shape
    (sum_check/benches/sum_check_benchmark.rs:9-31 — criterion over `prove` of a
    12-var random BN254 Fr MultilinearPoly): the reference-faithful C port
    (oracle/zk_oracle.c or_sumcheck_prove, one thread) as the median of `runs`
    proves after 10 warm-up, and the GPU library's `prove` on the same table."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle as co  # baseline/checker only

    import zk_amd

    evals = co.synth(field, 1, 0, 0, 1 << nvars)
    cpu = []
    for i in range(runs + 10):
        t0 = time.perf_counter()
        rp, cs = co.prove(field, evals)
        if i >= 10:
            cpu.append(time.perf_counter() - t0)
    poly = zk_amd.MultilinearPoly(evals, field, ctx)
    gpu = []
    for i in range(runs + 10):
        t0 = time.perf_counter()
        proof = zk_amd.prove(poly, ctx=ctx)
        if i >= 10:
            gpu.append(time.perf_counter() - t0)
    same = [v for p in proof.proof_polynomials for v in p] == co.from_limbs(rp.reshape(-1, 4)) \
        and proof.claimed_sum == cs
    cpu.sort()
    gpu.sort()
    ops = 6.0 * ((1 << nvars) - 1)
    return {
        "workload": f"sum_check prove, {nvars}-var BN254 Fr MultilinearPoly (seed 1), shape of "
        "sum_check_benchmark.rs:9-31",
        "cpu_port_median_us": cpu[len(cpu) // 2] * 1e6,
        "cpu_port_field_ops_per_s": ops / cpu[len(cpu) // 2],
        "cpu_cores": 1,
        "gpu_median_us": gpu[len(gpu) // 2] * 1e6,
        "runs": runs,
        "same_proof": bool(same),
        "note": "at 12 variables the GPU call is launch- and hand-off-bound (12 rounds, host transcript "
        "absorbs the 128 KiB table first); the GPU leg is for completeness, the CPU port is the config-1 number",
    }


def plain_bench(ctx, field: int, nvars: int, reps: int = 2) -> dict:
    """GPU plain `prove` / `verify` (sum_check_protocol.rs:25-84) at scale, from host
    tables (the ABI takes host evaluations), with the serial host Keccak absorb of
    the 32 N table bytes that the protocol starts with (:27, F6) timed on its own:
    it is the Amdahl floor of plain `prove` on any device."""
    import ctypes as C

    import zk_amd
    from zk_amd._lib import check, lib

    evals = ctx.synth(field, 1 << nvars, seed=1, table=0).download()  # canonical host limbs
    poly = zk_amd.MultilinearPoly(evals, field, ctx)
    out = (C.c_uint8 * 32)()
    ka = []
    for _ in range(reps):
        t0 = time.perf_counter()
        check(lib().zk_keccak256(evals.ctypes.data, evals.nbytes, out))
        ka.append(time.perf_counter() - t0)
    pv, vf = [], []
    ok = True
    for i in range(reps + 1):
        t0 = time.perf_counter()
        proof = zk_amd.prove(poly, ctx=ctx)
        t1 = time.perf_counter()
        ok = ok and zk_amd.verify(poly, proof, ctx=ctx)
        t2 = time.perf_counter()
        if i:
            pv.append(t1 - t0)
            vf.append(t2 - t1)
    med = lambda v: sorted(v)[len(v) // 2] * 1e3  # noqa: E731
    return {
        "workload": f"plain prove + verify, {nvars}-var BN254 Fr table from host memory ({evals.nbytes / 2**20:.0f} MiB)",
        "prove_ms": med(pv),
        "verify_ms": med(vf),
        "host_keccak_absorb_ms": med(ka),
        "absorb_share_of_prove": med(ka) / med(pv),
        "verified": bool(ok),
    }


def cpu_baseline(field: int, nvars: int, fast_nvars: int) -> dict:
    """Reference CPU path: the C restatement of the reference prover
    (oracle/zk_oracle.c, same algorithm and allocation pattern as
    sum_check_protocol.rs:86-166), single thread like the reference (no rayon),
    timed on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle as co  # checker/baseline only

    tabs = [co.synth(field, 3, t, 0, 1 << nvars) for t in range(4)]
    t0 = time.perf_counter()
    polys, chal = co.gkr_prove(field, tabs, co.Transcript())
    dt = time.perf_counter() - t0
    # the reference-faithful port's proof pins the committed full-size fixture
    # (written by the fused restatement): abort unless the two agree
    port_check = proof_digest_check(field, nvars, 3, polys, chal, abort=False)
    if port_check["matches_oracle_fixture"] is False:
        raise SystemExit(f"reference-faithful CPU port's proof digest {port_check['blob_keccak256']} != "
                         f"{port_check['fixture']}")
    ops = 32.0 * ((1 << nvars) - 1)
    del tabs
    # the fast restatement (fused, in place, OpenMP on every thread this
    # process may use) on the full workload: the best the host can do
    nf = fast_nvars
    ftabs = [co.synth(field, 3, t, 0, 1 << nf) for t in range(4)]
    t0 = time.perf_counter()
    co.gkr_prove(field, ftabs, co.Transcript(), fast=True)
    dtf = time.perf_counter() - t0
    del ftabs
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = list(range(os.cpu_count() or 1))
    return {
        "value": ops / dt,
        "unit": "field-ops/s",
        "cores": 1,
        "kind": "port",
        "nproc": os.cpu_count(),
        "affinity_cpus": len(aff),
        "affinity_mask": _ranges(aff),
        "sample": f"one gkr_prove over a {nvars}-var synthetic SumPoly (4 tables x 2^{nvars}), "
        f"{dt:.2f} s single-thread, host '{cpu_model()}' ({os.cpu_count()} logical CPUs)",
        "prover_ms_sample": dt * 1e3,
        "matches_fixture": port_check["matches_oracle_fixture"],
        "port_proof": port_check,
        "fast_allcores": {
            "value": 32.0 * ((1 << nf) - 1) / dtf,
            "unit": "field-ops/s",
            "cores": co.threads(),
            "kind": "port (fused OpenMP restatement, oracle/zk_oracle.c or_gkr_prove_fast)",
            "threads_note": "OpenMP threads = OMP_NUM_THREADS (the GPU box's CPU share per GPU is 16 of its "
            f"{os.cpu_count()} logical CPUs; affinity mask {_ranges(aff)}), so this is every thread the lease allows",
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "sample": f"one gkr_prove over {nf} vars (4 tables x 2^{nf}, same seed as the GPU run)",
            "prover_ms": dtf * 1e3,
        },
    }


def fold_bench(ctx, field: int, nvars: int = 20, reps: int = 10) -> dict:
    """BASELINE config 2: one partial_evaluate(0, r) of a 20-var table. 10
    distinct input/output buffer pairs (480 MiB > 256 MiB Infinity Cache) are
    rotated so every launch streams from HBM."""
    import ctypes as C

    import numpy as np

    from zk_amd._lib import check, lib
    from zk_amd.elems import as_limbs, ptr

    bufs = [(ctx.synth(field, 1 << nvars, seed=2, table=i), ctx.alloc(field, 1 << (nvars - 1))) for i in range(reps)]
    r = ptr(as_limbs([12345678901234567890]))
    for i, o in bufs[:2]:
        check(lib().zk_dev_mle_partial_evaluate(ctx.h, field, i.ptr, nvars, 0, 0, r, o.ptr))
    ctx.reset_stats()
    ctx.set_timing(True)
    for _ in range(3):
        for i, o in bufs:
            check(lib().zk_dev_mle_partial_evaluate(ctx.h, field, i.ptr, nvars, 0, 0, r, o.ptr))
    ctx.set_timing(False)
    k = ctx.stats()["kernels"]["fold"]
    gbs = k["alg_bytes"] / (k["ms"] / 1e3) / 1e9
    return {
        "workload": f"partial_evaluate(0, r), {nvars}-var BN254 Fr, {reps} rotated buffers",
        "launches": k["launches"],
        "avg_launch_us": k["ms"] * 1e3 / k["launches"],
        "bytes_per_launch": k["alg_bytes"] / k["launches"],
        "achieved_GBs": gbs,
        "frac_of_hbm_peak": gbs / HBM_PEAK_GBS,
    }


def serving_bench(field: int, tabs, n: int, ref_ch, streams: int = 2, per: int = 40) -> dict:
    """Serving shape, never `value`: `streams` independent proofs in flight on
    the one GPU — one host thread and one context (stream, pinned page,
    workspaces) each, the same device-resident tables (read only), fresh
    transcripts. One proof's tail (rounds 6-23, latency-bound) overlaps the
    other's large passes. Aggregate proofs/s and per-proof latency; every proof
    must equal the headline proof (tools/serve_streams.py sweeps the count)."""
    import ctypes as C
    import threading

    import numpy as np

    import zk_amd
    from zk_amd._lib import check, lib
    from zk_amd.elems import as_limbs, ptr

    arr = (C.c_void_p * 4)(*[t.ptr.value for t in tabs])
    zero = as_limbs([0])
    ctxs = [zk_amd.Context(tabs[0].ctx.device) for _ in range(streams)]
    lat = [[] for _ in range(streams)]
    ok = [True] * streams

    def prove(c, ch):
        coeffs = np.zeros((n, 3, 4), np.uint64)
        nco = np.zeros(n, np.uint8)
        tr = zk_amd.Transcript(field)
        check(lib().zk_dev_gkr_sumcheck_prove_sharded(c.h, field, arr, n, 0, ptr(zero), tr.h, ptr(coeffs), ptr(nco),
                                                      ptr(ch)))

    try:
        for c in ctxs:
            ch = np.zeros((n, 4), np.uint64)
            for _ in range(3):
                prove(c, ch)
        barrier = threading.Barrier(streams + 1)

        def run(i):
            ch = np.zeros((n, 4), np.uint64)
            barrier.wait()
            for _ in range(per):
                t0 = time.perf_counter()
                prove(ctxs[i], ch)
                lat[i].append(time.perf_counter() - t0)
                ok[i] = ok[i] and np.array_equal(ch, ref_ch)

        th = [threading.Thread(target=run, args=(i,)) for i in range(streams)]
        for t in th:
            t.start()
        barrier.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
    finally:
        for c in ctxs:
            c.close()
    alll = sorted(x for lt in lat for x in lt)
    if not all(ok):
        raise SystemExit("serving leg: a concurrent proof differs from the headline proof")
    total = streams * per
    return {"workload": f"{streams} independent {n}-var gkr_prove streams on one GPU (one context and host thread each, "
                        "shared read-only tables)",
            "proofs": total, "proofs_per_s": total / wall, "ms_per_proof_aggregate": wall * 1e3 / total,
            "field_ops_per_s": 32.0 * ((1 << n) - 1) * total / wall,
            "latency_ms_median": alll[len(alll) // 2] * 1e3, "latency_ms_p90": alll[int(len(alll) * 0.9)] * 1e3,
            "same_proof_as_headline": True}


def e2e_bench(ctx, field: int, tabs, n: int, reps: int = 3) -> dict:
    """The PCIe-inclusive rate (SURVEY.md 8(d) "end-to-end time including
    H2D"), never `value`: the same proof through the host-pointer ABI
    zk_gkr_sumcheck_prove, tables handed over in host memory in ark's
    Montgomery layout (what a Rust shim passes without conversion), uploaded by
    the library inside the call. Host buffers are ordinary pageable memory."""
    import ctypes as C

    import numpy as np

    import zk_amd
    from zk_amd._lib import check, lib
    from zk_amd.context import REPR_MONTGOMERY
    from zk_amd.elems import as_limbs, ptr

    host = [t.download(REPR_MONTGOMERY) for t in tabs]
    arr = (C.c_void_p * 4)(*[h.ctypes.data for h in host])
    coeffs = np.zeros((n, 3, 4), np.uint64)
    nco = np.zeros(n, np.uint8)
    ch = np.zeros((n, 4), np.uint64)
    cs = np.zeros((1, 4), np.uint64)
    zero = as_limbs([0])
    times = []
    for i in range(reps + 1):
        tr = zk_amd.Transcript(field)
        t0 = time.perf_counter()
        check(lib().zk_gkr_sumcheck_prove(ctx.h, field, REPR_MONTGOMERY, arr, n, ptr(zero), tr.h, ptr(coeffs),
                                          ptr(nco), ptr(ch), ptr(cs)))
        if i:
            times.append(time.perf_counter() - t0)
    times.sort()
    gib = 4 * (1 << n) * 32
    return {
        "workload": f"zk_gkr_sumcheck_prove from host memory, {n} vars, 4 tables x 2^{n} ({gib / 2**30:.0f} GiB)",
        "ms_median": times[len(times) // 2] * 1e3,
        "upload_GBs_effective": gib / times[len(times) // 2] / 1e9,
        # outputs follow the input repr (Montgomery); canonical for the caller's comparison
        "challenges": ctx.upload(field, ch, REPR_MONTGOMERY).download(),
    }


def circuit_bench(ctx, field: int, log_inputs: int = 12, reps: int = 7) -> dict:
    """a full GKR prove over a random binary-tree circuit with
    2^log_inputs inputs — circuit evaluation, every layer's two-phase sum-check
    over tables of 2G entries (sparse wiring) on the device, transcript on the
    host. The input layer's sum-check runs over 2*log_inputs variables (24 at
    the default); ZK_CIRCUIT_DENSE=1 builds the dense (2G)^2 tables instead."""
    import random

    import zk_amd
    from zk_amd.gkr import Circuit, Operation, prove, verify

    rng = random.Random(11)
    structure = [[rng.choice((Operation.Add, Operation.Mul)) for _ in range(1 << (log_inputs - 1 - i))]
                 for i in range(log_inputs)]
    p = zk_amd.modulus(field)
    inputs = [rng.randrange(p) for _ in range(1 << log_inputs)]
    circ = Circuit(structure, field)
    from zk_amd.elems import as_limbs

    x = as_limbs(inputs)  # the C ABI's element layout (uint64[n, 4]), as a Rust caller holds Vec<Fr>
    proof = prove(circ, x, ctx)  # warm-up
    ok = verify(proof, circ, inputs) and prove(circ, inputs, ctx).random_challenges == proof.random_challenges
    times, times_int = [], []
    for _ in range(reps):  # wall time of the API call, no events
        t0 = time.perf_counter()
        prove(circ, x, ctx)
        times.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        prove(circ, inputs, ctx)  # the same with Python-int inputs (adds their conversion)
        times_int.append(time.perf_counter() - t0)
    ctx.reset_stats()  # one more proof with HIP events on the layer kernels
    ctx.set_timing_kinds(["layer"])
    prove(circ, inputs, ctx)
    ctx.set_timing(False)
    k = ctx.stats()["kernels"]["layer"]
    times.sort()
    times_int.sort()
    return {
        "workload": f"gkr::prove over a random {log_inputs}-layer binary-tree circuit, {1 << log_inputs} inputs "
                    f"(input-layer sum-check over {2 * log_inputs} variables), {'BN254 Fr' if field == 0 else field}",
        "ms_median": times[len(times) // 2] * 1e3,
        "inputs": "uint64[n, 4] limb array (the C ABI layout)",
        "ms_median_python_int_inputs": times_int[len(times_int) // 2] * 1e3,
        "verified": ok,
        "reps": reps,
        "layer_kernels_ms_per_proof": k["ms"],
        "layer_prover": "dense (2G)^2 tables" if os.environ.get("ZK_CIRCUIT_DENSE", "0") not in ("", "0")
        else "two phases over tables of 2G entries",
        "note": "the reference builds add_i/mul_i densely (2^(3g+2) entries: 2^35 at this size) and cannot run it",
    }


def circuit_kzg_bench(ctx, log_inputs: int = 14, reps: int = 5) -> dict:
    """gkr::prove WITH the input layer's KZG step (gkr_protocol.rs:92-118;
    zk_gkr_circuit_prove_kzg) over BLS12-381 Fr at the largest circuit the
    layered prover takes (2^14 inputs): circuit GKR + KZG setup over 14
    variables + commit + two get_proofs; gkr::verify (with both KZG pairings
    checks, no inputs) must accept it."""
    import random

    import zk_amd
    from zk_amd.gkr import Circuit, Operation, prove, verify
    from zk_amd.elems import as_limbs

    field = 2
    rng = random.Random(14)
    structure = [[rng.choice((Operation.Add, Operation.Mul)) for _ in range(1 << (log_inputs - 1 - i))]
                 for i in range(log_inputs)]
    p = zk_amd.modulus(field)
    x = as_limbs([rng.randrange(p) for _ in range(1 << log_inputs)])
    taus = [rng.randrange(p) for _ in range(log_inputs)]
    circ = Circuit(structure, field)
    proof = prove(circ, x, ctx, taus=taus)  # warm-up (and the setup's tables)
    ok = verify(proof, circ)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        prove(circ, x, ctx, taus=taus)
        times.append(time.perf_counter() - t0)
    times.sort()
    return {"workload": f"gkr::prove with the input layer's KZG (setup, commit, 2 get_proofs over {log_inputs} "
                        f"variables), random {log_inputs}-layer circuit, {1 << log_inputs} inputs, BLS12-381 Fr",
            "ms_median": times[len(times) // 2] * 1e3, "reps": reps, "verified": bool(ok)}


def config5_bench(ctx, nvars: int = 24, reps: int = 3) -> dict:
    """BASELINE config 5: the 24-variable GKR sum-check over BLS12-381 Fr, and
    the KZG commitment of a 24-variable MLE over BLS12-381
    G1: a 2^24-point Pippenger MSM against the Lagrange basis of fixed taus."""
    import ctypes as C
    import random

    import numpy as np

    import zk_amd
    from zk_amd._lib import check, lib
    from zk_amd.elems import as_limbs, ptr
    from zk_amd.kzg import KZG

    field = 2
    tabs = [ctx.synth(field, 1 << nvars, seed=5, table=t) for t in range(4)]
    arr = (C.c_void_p * 4)(*[t.ptr.value for t in tabs])
    coeffs = np.zeros((nvars, 3, 4), np.uint64)
    nco = np.zeros(nvars, np.uint8)
    ch = np.zeros((nvars, 4), np.uint64)
    zero = ptr(as_limbs([0]))

    def gkr():
        tr = zk_amd.Transcript(field)
        check(lib().zk_dev_gkr_sumcheck_prove_sharded(ctx.h, field, arr, nvars, 0, zero, tr.h, ptr(coeffs), ptr(nco),
                                                      ptr(ch)))

    gkr()
    ts = []
    for _ in range(5 * reps):  # (the proof is ~1 ms: more samples than the commits)
        t0 = time.perf_counter()
        gkr()
        ts.append(time.perf_counter() - t0)
    gkr_ms = sorted(ts)[len(ts) // 2] * 1e3
    del tabs
    rng = random.Random(55)
    taus = [rng.randrange(zk_amd.modulus(field)) for _ in range(nvars)]
    t0 = time.perf_counter()
    k = KZG(taus, ctx)
    setup_ms = (time.perf_counter() - t0) * 1e3
    evals = ctx.synth(field, 1 << nvars, seed=5, table=0)
    out = np.zeros((1, 12), np.uint64)
    check(lib().zk_dev_kzg_commit(ctx.h, k.h, evals.ptr, ptr(out)))  # warm-up
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        check(lib().zk_dev_kzg_commit(ctx.h, k.h, evals.ptr, ptr(out)))
        ts.append(time.perf_counter() - t0)
    commit_ms = sorted(ts)[reps // 2] * 1e3
    commit_check = kzg_commit_check(nvars, out)
    # KZG::get_proof (kzg.rs:59-95) of the same MLE at a random point: nvars
    # quotient commitments (MSMs of 2^(nvars-1) .. 1 points), the evaluations
    # resident in HBM like the commit's (zk_dev_kzg_get_proof; median of reps
    # after a warm-up), and once from host memory (zk_kzg_get_proof: the 512 MiB
    # upload inside the time); both checked by KZG::verify's pairings (host,
    # kzg.rs:97-129) and equal
    from zk_amd.context import REPR_CANONICAL
    from zk_amd.kzg import _points

    host = evals.download()  # canonical limbs
    point = [rng.randrange(zk_amd.modulus(field)) for _ in range(nvars)]
    pt = as_limbs(point)
    v = np.zeros((1, 4), np.uint64)
    check(lib().zk_mle_evaluate(ctx.h, field, REPR_CANONICAL, ptr(host), nvars, ptr(pt), nvars, ptr(v)))
    prf = np.zeros((nvars, 12), np.uint64)
    check(lib().zk_dev_kzg_get_proof(ctx.h, k.h, REPR_CANONICAL, evals.ptr, ptr(v), ptr(pt), ptr(prf)))  # warm-up
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        check(lib().zk_dev_kzg_get_proof(ctx.h, k.h, REPR_CANONICAL, evals.ptr, ptr(v), ptr(pt), ptr(prf)))
        ts.append(time.perf_counter() - t0)
    proof_ms = sorted(ts)[reps // 2] * 1e3
    prf_host = np.zeros((nvars, 12), np.uint64)
    t0 = time.perf_counter()
    check(lib().zk_kzg_get_proof(ctx.h, k.h, REPR_CANONICAL, ptr(host), ptr(v), ptr(pt), ptr(prf_host)))
    proof_host_ms = (time.perf_counter() - t0) * 1e3
    if not np.array_equal(prf, prf_host):
        raise SystemExit("KZG get_proof: the device-resident and host-input proofs differ")
    t0 = time.perf_counter()
    proof_ok = KZG.verify(_points(out)[0], int(sum(int(v[0, i]) << (64 * i) for i in range(4))), _points(prf), point,
                          k.g2_taus)
    verify_ms = (time.perf_counter() - t0) * 1e3
    if not proof_ok:
        raise SystemExit("KZG get_proof at full size did not verify")
    k.close()
    del host
    # a second setup (other taus) on the same context: its fixed-base table and
    # scratch buffers already exist, so this is the steady-state cost of a setup
    t0 = time.perf_counter()
    k2 = KZG([rng.randrange(zk_amd.modulus(field)) for _ in range(nvars)], ctx)
    setup_warm_ms = (time.perf_counter() - t0) * 1e3
    k2.close()
    n = 1 << nvars
    return {
        "workload": f"BLS12-381: gkr_prove over {nvars} variables (A*S + M*P, seed 5) and the KZG commitment of a "
                    f"{nvars}-variable MLE (2^{nvars}-point G1 MSM, Lagrange basis of fixed taus)",
        "gkr_prove_ms": gkr_ms,
        "gkr_field_ops_per_s": 32.0 * (n - 1) / (gkr_ms / 1e3),
        "kzg_setup_ms": setup_ms,
        "kzg_setup_warm_ms": setup_warm_ms,
        "kzg_commit_ms": commit_ms,
        "msm_points_per_s": n / (commit_ms / 1e3),
        "commit_check": commit_check,
        "kzg_get_proof_ms": proof_ms,
        "kzg_get_proof_host_input_ms": proof_host_ms,
        "kzg_get_proof_note": f"{nvars} quotient commitments (MSMs of 2^{nvars - 1} .. 1 points) + folds, evaluations "
                              f"resident in HBM (zk_dev_kzg_get_proof, median of {reps}); host_input: from host memory "
                              "(zk_kzg_get_proof, the 512 MiB upload inside the time), the same proof; verified by "
                              "KZG::verify's pairings",
        "kzg_get_proof_verified": bool(proof_ok),
        "kzg_verify_host_ms": verify_ms,
        "note": "the reference commits with a naive sum of 2^24 full scalar multiplications (kzg.rs:131-144)",
    }


def config4_bench(ctx, field: int, world: int, rank: int, barrier, total_nvars: int = 26, reps: int = 15) -> dict:
    """BASELINE config 4 exactly: one gkr_prove over `total_nvars` variables
    in total, the hypercube split over all ranks (each holds 2^(total - log2 G)
    elements per table; strong scaling, beside the weak-scaling headline).
    Every rank calls it (the proof runs the per-round all-reduce); max over
    ranks of the median per-proof time, barrier-bracketed."""
    import ctypes as C

    import numpy as np
    import torch
    import torch.distributed as dist

    import zk_amd
    from zk_amd._lib import check, lib
    from zk_amd.elems import as_limbs, ptr

    lg = (world - 1).bit_length()
    nloc = total_nvars - lg
    tabs = [ctx.synth(field, 1 << nloc, seed=4, table=t, index0=rank, stride=world) for t in range(4)]
    arr = (C.c_void_p * 4)(*[t.ptr.value for t in tabs])
    coeffs = np.zeros((total_nvars, 3, 4), np.uint64)
    nco = np.zeros(total_nvars, np.uint8)
    ch = np.zeros((total_nvars, 4), np.uint64)
    zero = ptr(as_limbs([0]))
    times = []
    for i in range(reps + 3):  # 3 warm-up proofs (the first allocates the 26-variable workspace)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr = zk_amd.Transcript(field)
        check(lib().zk_dev_gkr_sumcheck_prove_sharded(ctx.h, field, arr, nloc, 0, zero, tr.h, ptr(coeffs), ptr(nco),
                                                      ptr(ch)))
        torch.cuda.synchronize()
        if i >= 3:
            times.append(time.perf_counter() - t0)
    # one more proof with HIP events on every launch (its times are reported,
    # not counted in ms_median): where the proof's time goes
    ctx.reset_stats()
    ctx.set_timing_kinds(["gkr_round0", "gkr_round", "gkr_round_lanes", "gkr_tail", "gkr_dround", "gkr_dtail", "gkr_d0",
                          "gkr_dm", "gkr_t33", "coll"])
    barrier()
    tr = zk_amd.Transcript(field)
    check(lib().zk_dev_gkr_sumcheck_prove_sharded(ctx.h, field, arr, nloc, 0, zero, tr.h, ptr(coeffs), ptr(nco),
                                                  ptr(ch)))
    ctx.set_timing(False)
    launches = ctx.launches()
    ctx.reset_stats()
    for t in tabs:
        t.free()
    digest = proof_check(field, total_nvars, 4, coeffs, nco, ch)
    times.sort()
    med = times[len(times) // 2]
    if world > 1:
        t = torch.tensor([med], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        med = float(t.item())
    return {
        "workload": f"gkr_prove over {total_nvars} variables total ({nloc} per GPU), seed 4, split over {world} GPU(s)",
        "scaling": "strong",
        "ms_median": med * 1e3,
        "ms_min": times[0] * 1e3,
        "ms_max": times[-1] * 1e3,
        "proofs_timed": reps,
        "field_ops_per_s": 32.0 * ((1 << total_nvars) - 1) / med,
        "launches_of_proof": [{"kind": x["kind"], "us": round(x["ms"] * 1e3, 1), "alg_GB": round(x["alg_bytes"] / 1e9, 4)}
                              for x in launches],
        "challenge0_lo": int(ch[0, 0]),
        "proof": digest,
    }


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, cmd: list, env_extra: dict | None = None, grace_s: float = 10.0,
                poll_s: float = 0.2, timeout_s: float | None = None) -> tuple[int, str]:
    """Launcher for `bench.py --gpus N` run without torch.distributed.run: start
    `cmd` as N fresh child processes, one per GPU, with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (what torchrun would set), and
    wait for all of them. The caller (the parent) never imports torch or touches
    the GPU: it is a launcher, not a re-exec. Rank 0's stdout is captured
    (the bench's one JSON line); every other stream goes to the parent's stderr.
    When a rank exits non-zero the others are given `grace_s` to finish, then
    killed (their peers would otherwise wait at a barrier). Returns (exit code,
    rank 0's stdout): 0 only if every rank exited 0, else the first failing
    rank's code (a signal death maps to 128 + signal). With `timeout_s`, ranks
    still running after it are killed and the result is a failure (124)."""
    import signal

    # (a caller that is itself a torch.distributed.run worker — rank 0 starting
    # the peer-reduction side leg — must not hand its elastic-agent settings
    # down: with TORCHELASTIC_USE_AGENT_STORE the children would wait for an
    # agent store on their fresh port instead of hosting their own)
    drop = ("TORCHELASTIC_", "GROUP_", "ROLE_", "TORCH_ELASTIC")
    env0 = {k: v for k, v in os.environ.items() if not k.startswith(drop)}
    env0.update({"WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                 "MASTER_PORT": str(_free_port()), "ZK_BENCH_LAUNCHER": "self"})
    env0.update(env_extra or {})
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
        procs.append(subprocess.Popen(cmd, env=env, stdin=subprocess.DEVNULL,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(),
                                      start_new_session=True))
    import threading

    out0 = []
    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    first_bad, t_bad = None, None
    t_start = time.monotonic()
    while True:
        codes = [p.poll() for p in procs]
        if timeout_s is not None and first_bad is None and time.monotonic() - t_start > timeout_s \
                and any(c is None for c in codes):
            print(f"bench launcher: ranks still running after {timeout_s:.0f} s", file=sys.stderr)
            first_bad, t_bad = -1, time.monotonic() - grace_s - 1  # kill now
            continue
        if first_bad is None:
            for r, c in enumerate(codes):
                if c is not None and c != 0:
                    first_bad, t_bad = r, time.monotonic()
                    print(f"bench launcher: rank {r} exited with {c}", file=sys.stderr)
                    break
        if all(c is not None for c in codes):
            break
        if first_bad is not None and time.monotonic() - t_bad > grace_s:
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)  # the rank's own session (start_new_session)
                    except ProcessLookupError:
                        pass
            for p in procs:
                p.wait()
            break
        time.sleep(poll_s)
    reader.join(timeout=30)
    text = out0[0].decode(errors="replace") if out0 and out0[0] else ""
    codes = [p.returncode for p in procs]
    if first_bad is None:
        bad = [c for c in codes if c != 0]
        rc = bad[0] if bad else 0
    elif first_bad < 0:
        rc = 124
    else:
        rc = codes[first_bad]
    if rc < 0:
        rc = 128 - rc
    return rc, text


def main() -> None:
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # self-launch: N fresh rank processes of this script (the parent never
        # imports torch or touches a GPU); rank 0's JSON line is relayed
        rc, text = spawn_ranks(args.gpus, [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:])
        lines = [ln for ln in text.splitlines() if ln.strip()]
        if rc == 0 and lines:
            sys.stdout.write(lines[-1] + "\n")
            sys.stdout.flush()
        elif rc == 0:
            print("bench launcher: rank 0 printed no result line", file=sys.stderr)
            rc = 1
        raise SystemExit(rc)
    # stdout carries exactly ONE line, the JSON result: libraries that print
    # banners to stdout (RCCL's "RCCL version ..." at communicator init) are
    # sent to stderr by pointing fd 1 there; the result goes to the saved fd.
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N ranks (torch.distributed.run "
                         "--nproc-per-node N, or plain `python bench.py --gpus N`, which starts them itself)")
    field = FIELDS[args.field]

    import ctypes as C

    import numpy as np
    import torch
    import torch.distributed as dist

    import zk_amd
    from zk_amd._lib import check, lib
    from zk_amd.context import rccl_unique_id
    from zk_amd.elems import as_limbs, ptr

    if args.comm == "host":
        # (the library launches each step after its challenge with a host
        # all-reduce, so ranks that share a card cannot starve each other)
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if args.force_rccl and world == 1:
        os.environ["ZK_FORCE_COLLECTIVES"] = "1"  # read at zk_ctx_create
    ctx = zk_amd.Context(local)
    if args.force_rccl and world == 1:
        ctx.attach_rccl(0, 1, rccl_unique_id())
        if args.reduce == "peer":
            ctx.attach_peer_reduce()
    lg = (world - 1).bit_length()
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        import datetime

        # (a rank that fails leaves the others at a barrier: fail within minutes, not torch's 30)
        dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=10))
        if args.comm == "host":
            from zk_amd.dist import TorchAllreduce

            ctx.attach_host_comm(rank, world, TorchAllreduce())
        else:
            obj = [rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            ctx.attach_rccl(rank, world, obj[0])
        if args.reduce == "peer":
            ctx.attach_peer_reduce()  # collective; checked across the world, raises if it fails

    nloc = args.nvars
    n = nloc + lg
    # this rank's shard: local m <-> global m*world + rank
    tabs = [ctx.synth(field, 1 << nloc, seed=args.seed, table=t, index0=rank, stride=world) for t in range(4)]
    arr = (C.c_void_p * 4)(*[t.ptr.value for t in tabs])
    coeffs = np.zeros((n, 3, 4), np.uint64)
    nco = np.zeros(n, np.uint8)
    ch = np.zeros((n, 4), np.uint64)
    zero = ptr(as_limbs([0]))

    def step():
        tr = zk_amd.Transcript(field)
        check(lib().zk_dev_gkr_sumcheck_prove_sharded(ctx.h, field, arr, nloc, 0, zero, tr.h, ptr(coeffs), ptr(nco),
                                                      ptr(ch)))

    def barrier():
        if world > 1:
            dist.barrier()

    step()  # the first proof, checked against the full-size oracle fixture
    digest = proof_check(field, n, args.seed, coeffs, nco, ch)
    for _ in range(args.warmup):
        step()
    first_challenges = ch.copy()
    ctx.reset_stats()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == args.steps - 1:
            # HIP events ride on the dispatch packets of the dominant kernel
            # (hipExtLaunchKernelGGL start/stop events on the launch stream)
            # during the LAST timed step only: their marker packets cost the GPU
            # ~5 us per round, so timing every step would inflate ms_per_step
            st0 = ctx.stats()
            ctx.set_timing_kinds([] if args.no_events else ["gkr_round0", "gkr_round", "gkr_round_lanes", "gkr_tail", "gkr_dround", "gkr_dtail", "gkr_d0", "gkr_dm", "gkr_t33", "coll"])
        step()
    torch.cuda.synchronize()
    local_s = time.perf_counter() - t0  # this rank's own time, before the closing barrier
    barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_timing(False)
    st = ctx.stats()
    launches = ctx.launches()
    ranks = None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # per rank (SCALE attribution): its own time before the closing barrier,
        # the host's wait for round results, the collectives (count, and the
        # time of the last timed proof's: RCCL events on the stream or the host
        # communicator's callback wall time)
        coll_ms = sum(x["ms"] for x in launches if x["kind"] == "coll")
        mine = {"rank": rank, "own_ms_per_step": local_s * 1e3 / args.steps,
                "host_wait_ms_per_step": st["host_wait_us"] / 1e3 / args.steps,
                "host_work_ms_per_step": st["host_work_us"] / 1e3 / args.steps,
                "collectives_per_step": st["collectives"] / args.steps,
                "collective_ms_last_step": coll_ms,
                "collective_launches_last_step": sum(1 for x in launches if x["kind"] == "coll")}
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    assert np.array_equal(first_challenges, ch), "proof changed between steps"

    ops = 32.0 * ((1 << n) - 1) * args.steps
    value = ops / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    k = st["kernels"]
    # per kernel kind over the event-timed (last) step; the dominant kernel is
    # the kind with the most time in the proof (k_gkr_dm at n = 24)
    def kind(name):
        d = {f: k[name][f] - st0["kernels"][name][f] for f in ("launches", "alg_bytes")}
        d["ms"] = k[name]["ms"]
        return d

    round_kinds = {
        "gkr_d0": "k_gkr_d0t (rounds 0-2 in one pass over the input tables: 27 moment sums of corner-pair "
                  "products on the int8 matrix cores, nothing written; k_gkr_d0m for rounds 0-1 when n < 11)",
        "gkr_t33": "k_gkr_t33 (fold the level-(i-3) tables by three challenges on the int8 matrix cores, write "
                   "level i, rounds i..i+2 as 27 moment sums)",
        "gkr_dm": "k_gkr_dm3 / k_gkr_dm (fold by three / two challenges on the int8 matrix cores, write level i, "
                  "eight grid-point product sums of rounds i, i+1)",
        "gkr_round0": "k_gkr_round0 (round 0: e0, e1, e2 over the input tables)",
        "gkr_round": "k_gkr_round (round 1: fold by r0 + round sums)",
        "gkr_round_lanes": "k_gkr_round_lanes (single small rounds, 8 lanes per pair)",
        "gkr_dround": "k_gkr_dround (two rounds per launch: pending folds + round m sums + round m+1 quadratics)",
        "gkr_dtail": "k_gkr_dtail (the small double steps in one persistent kernel; host hand-offs included)",
        "gkr_tail": "k_gkr_tail (ZK_DROUND=0: small single rounds in one persistent kernel)",
    }
    per_kind = {}
    for name, desc in round_kinds.items():
        d = kind(name)
        if d["launches"]:
            per_kind[name] = {"kernel": desc, "launches": d["launches"], "ms": d["ms"],
                              "alg_GB": d["alg_bytes"] / 1e9,
                              "achieved_GBs": d["alg_bytes"] / (d["ms"] / 1e3) / 1e9 if d["ms"] else None}
    # the dominant kernel: the longest launch of the timed proof (k_gkr_t33 over
    # the input tables at n = 24: rounds 3-5); collectives are listed apart
    colls = [x for x in launches if x["kind"] == "coll"]
    launches = [x for x in launches if x["kind"] != "coll"]
    # --no-events: no launch was timed; the roofline fields then read 0
    top = max(launches, key=lambda x: x["ms"]) if launches else {"kind": "none", "ms": 0.0, "alg_bytes": 0.0}
    dom = top["kind"]
    all_b = sum(kind(nm)["alg_bytes"] for nm in per_kind)
    all_ms = sum(kind(nm)["ms"] for nm in per_kind)
    achieved = top["alg_bytes"] / (top["ms"] / 1e3) / 1e9 if top["ms"] else 0.0
    kernel_ms = sum(v["ms"] for kk, v in k.items() if kk != "coll")  # the timed (last) step
    muls = sum(v["field_muls"] for v in k.values()) / args.steps

    traffic, traffic_src = None, None
    import glob
    import re

    # the newest round's PMC traffic file (profiles/r<N>_traffic.json, tools/pmc_traffic.py)
    # (r6f_traffic.json: round 6's last tree, after r6_traffic.json)
    tfiles = sorted((f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json"))
                     if re.match(r"r\d+[a-z]*_traffic\.json$", os.path.basename(f))),
                    key=lambda f: (int(re.match(r"r(\d+)", os.path.basename(f)).group(1)), os.path.basename(f)))
    tpath = tfiles[-1] if tfiles else ""
    if os.path.exists(tpath) and n == 24:
        t = json.load(open(tpath))
        if t.get("kind") == dom and field == 0:  # the longest launch of this workload
            traffic = t["traffic_bytes_per_launch"]  # HBM bytes per launch, beside alg_bytes_per_launch
            traffic_src = f"profiles/{os.path.basename(tpath)} ({t['method']}); traffic/alg = {t['traffic_over_alg']:.4f}"
    cfg4 = config4_bench(ctx, field, world, rank, barrier) if args.config4 else None
    peer_leg = None
    if world > 1 and args.reduce == "comm" and not args.no_peer_leg:
        # the headline again with --reduce peer, in N fresh ranks that rank 0
        # starts as child processes (one per GPU): a failure or hang there can
        # only cost the side field, never this line
        if rank == 0:
            cmd = [sys.executable, "-u", os.path.abspath(__file__), "--gpus", str(world), "--steps", str(args.steps),
                   "--warmup", str(args.warmup), "--nvars", str(args.nvars), "--field", args.field, "--seed",
                   str(args.seed), "--comm", args.comm, "--reduce", "peer", "--no-config4", "--no-peer-leg"]
            t_leg = time.perf_counter()
            rc, text = spawn_ranks(world, cmd, timeout_s=180.0)
            lines = [ln for ln in text.splitlines() if ln.strip()]
            peer_leg = {"cmd": " ".join(cmd[2:]), "rc": rc, "wall_s": round(time.perf_counter() - t_leg, 1)}
            if rc == 0 and lines:
                try:
                    r = json.loads(lines[-1])
                    peer_leg.update({"value": r["value"], "ms_per_step": r["ms_per_step"], "proof": r["proof"],
                                     "reduce": r.get("reduce"), "comm": r.get("comm"),
                                     "collectives_per_step": r["breakdown_per_step"]["collectives"],
                                     "launches_of_proof": r["roofline"]["launches_of_proof"],
                                     "vs_comm_reduce": r["value"] / value})
                except (ValueError, KeyError) as e:
                    peer_leg["error"] = f"unreadable result line: {e}"
            else:
                peer_leg["error"] = "the peer-reduction ranks failed (their stderr is in this run's log)"
        barrier()
    comm = ctx.comm_info()  # what the attached communicator reports (RCCL: ncclCommCount / ncclCommUserRank)
    if comm["kind"] != "none" and (comm["count"] != world or comm["rank"] != rank):
        raise SystemExit(f"communicator reports rank {comm['rank']} of {comm['count']}, expected {rank} of {world}")
    if rank == 0:
        out = {
            "metric": "GKR sum-check field-ops/sec + prover ms, 24-var BN254, 1/2/4/8 GPU",
            "value": value,
            "unit": "field-ops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u256 mod p (8x32-bit Montgomery limbs)",
            "data": "synthetic (counter-based SplitMix64 tables mod p, device-generated; no dataset)",
            "config": {
                "workload": f"gkr_prove over SumPoly[A*S + M*P], {n} variables total "
                f"({nloc} per GPU), {args.field}, seed {args.seed}, tables resident in HBM",
                "field": args.field,
                "nvars_total": n,
                "nvars_per_gpu": nloc,
                "parallelism": f"hypercube split over {world} GPU(s) by low index bits; "
                + ("the step kernels sum the step's limb sums (<= 243 x u64) across ranks through IPC-mapped peer "
                   "buffers, one exchange per step of 2-3 rounds" if ctx.peer_reduce else
                   "1 RCCL all-reduce of the step's limb sums (<= 243 x u64) per step of 2-3 rounds" if args.comm == "rccl" else
                   "host (gloo) all-reduce per round: diagnostic, not the product path") if world > 1 else "single GPU",
            },
            "proof": digest,
            "comm": comm,
            "reduce": ("peer" if ctx.peer_reduce else "rccl" if comm["kind"] == "rccl" else comm["kind"])
            if comm["kind"] != "none" else None,
            "rccl_ranks": comm["count"] if comm["kind"] == "rccl" else None,
            "launcher": os.environ.get("ZK_BENCH_LAUNCHER", "torchrun" if world > 1 else "none"),
            "roofline": {
                "bound": "hbm",
                "kernel": round_kinds.get(dom, dom) + "; the longest launch of the proof",
                "bound_note": "HBM: the field products and folds run on the int8 matrix cores (DESIGN.md section 3a); "
                "k_gkr_d0t streams the inputs at 5.8-5.9 TB/s, reads only",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "launches": 1,
                "avg_launch_us": top["ms"] * 1e3,
                "alg_bytes_per_launch": top["alg_bytes"],
                "alg_GB_per_launch": top["alg_bytes"] / 1e9,
                "launches_of_proof": [{"kind": x["kind"], "us": round(x["ms"] * 1e3, 1),
                                       "alg_GB": round(x["alg_bytes"] / 1e9, 4)} for x in launches],
                "round_kernels": per_kind,
                "all_rounds_GBs": all_b / (all_ms / 1e3) / 1e9 if all_ms else None,
            },
            "breakdown_per_step": {
                "wall_ms": ms_per_step,
                "timed_kernel_ms": kernel_ms,
                "kernel_ms_by_kind": {kk: v["ms"] for kk, v in k.items() if v["ms"]},
                "host_syncs": st["host_syncs"] / args.steps,
                "host_wait_ms": st["host_wait_us"] / 1e3 / args.steps,
                "host_work_ms": st["host_work_us"] / 1e3 / args.steps,
                "collectives": st["collectives"] / args.steps,
                "field_muls": muls,
                "launches_by_kind": {kk: v["launches"] / args.steps for kk, v in k.items() if v["launches"]},
            },
        }
        if ranks is not None:
            own = [r["own_ms_per_step"] for r in ranks]
            out["multi_rank"] = {
                "note": "per rank over the timed steps; own_ms = a rank's time before the closing barrier, skew = "
                        "max - min of it; collective_ms = the collectives of the last timed proof (RCCL: HIP events "
                        "around each ncclAllReduce / ncclAllGather on the proof's stream; host communicator: the "
                        "callback's wall time)",
                "barrier_skew_ms_per_step": max(own) - min(own),
                "collective_ms_per_proof_max": max(r["collective_ms_last_step"] for r in ranks),
                "collective_us_each_rank0": [round(x["ms"] * 1e3, 2) for x in colls],
                "ranks": ranks,
            }
        if cfg4 is not None:
            out["config4_26var"] = cfg4
        if peer_leg is not None:
            out["peer_reduce_leg"] = peer_leg
        if not args.no_serving and world == 1:
            out["serving_2_streams"] = serving_bench(field, tabs, n, first_challenges)
        if not args.no_e2e and world == 1:
            e2e = e2e_bench(ctx, field, tabs, n)
            e2e["same_proof_as_device_resident"] = bool(np.array_equal(e2e.pop("challenges"), ch))
            out["e2e_host_tables"] = e2e
        if not args.no_fold and world == 1:
            out["fold_20var"] = fold_bench(ctx, field)
        if not args.no_circuit and world == 1:
            out["gkr_circuit"] = circuit_bench(ctx, field)
        if not args.no_config5 and world == 1:
            out["config5_bls12_381"] = config5_bench(ctx)
            out["gkr_circuit_kzg"] = circuit_kzg_bench(ctx)
        if not args.no_plain and world == 1:
            out["config1_12var_prove"] = config1_bench(ctx, field)
            out["plain_sumcheck"] = [plain_bench(ctx, field, nv) for nv in (20, 24)]
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(field, args.cpu_sample_nvars, args.cpu_fast_nvars)
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu_baseline"] = value / cb["value"]
        os.write(result_fd, (json.dumps(out) + "\n").encode())
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
