"""Sharded (multi-rank) GKR sum-check on the GPU through the C ABI.

Ranks are separate processes sharing the box's single GPU; their round sums
meet through the host all-reduce callback over gloo (RCCL refuses two ranks
on one device). The RCCL data path itself runs at world 1 with
ZK_FORCE_COLLECTIVES=1, which routes every round through ncclAllReduce and
the publish kernel. Every rank's proof must equal the oracle's single-process
proof over the full tables.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

import coracle as co
import gkr_schedule
import pyoracle as po

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "sharded_worker.py")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world: int, comm: str, field: int, nloc: int, out: str, extra_env=None) -> list[dict]:
    port = _free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), MASTER_PORT=str(port), COMM=comm,
                   FIELD=str(field), NLOCAL=str(nloc), OUT=out, MASTER_ADDR="127.0.0.1", **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, WORKER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        o, _ = p.communicate(timeout=240)
        logs.append(o.decode(errors="replace"))
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    res = []
    for rank in range(world):
        with open(os.path.join(out, f"rank{rank}.json")) as fh:
            res.append(json.load(fh))
    return res


def _oracle(field: int, n: int) -> dict:
    tabs = [co.synth(field, 19, t, 0, 1 << n) for t in range(4)]
    polys, chal = co.gkr_prove(field, tabs, co.Transcript())
    return {"polys": [[hex(x) for x in p] for p in polys], "chal": [hex(x) for x in chal],
            "blob_keccak": po.keccak256(po.proof_blob(po.BLOB_GKR, field, 0, [list(p) for p in polys])).hex()}


# the schedule (steps, gather boundary, collective count) the library builds
_bounds, _collectives = gkr_schedule.bounds, gkr_schedule.collectives


# (2, 20, 0): each rank's first kernel fills the card (512 blocks) while the
# other rank shares it: with pre-enqueued kernels spinning on their challenges
# this starved the other rank; the library launches step by step under a host
# communicator (host.hpp prelaunch()).
@pytest.mark.parametrize("world,nloc,field", [(2, 12, 0), (4, 9, 2), (2, 0, 1), (2, 5, 0), (2, 11, 1), (2, 14, 2),
                                              (2, 20, 0)])
def test_host_comm_ranks_match_single_process(tmp_path, world, nloc, field):
    res = _run(world, "host", field, nloc, str(tmp_path))
    want = _oracle(field, nloc + world.bit_length() - 1)
    for rank, r in enumerate(res):
        assert {"polys": r["polys"], "chal": r["chal"]} == {"polys": want["polys"], "chal": want["chal"]}, f"rank {rank}"
        # f4: the whole proof as one digest, identical on every rank and to the CPU oracle's
        assert r["blob_keccak"] == want["blob_keccak"], f"rank {rank}"
        assert r["collectives"] == _collectives(nloc)  # one all-reduce per step until the gather, then the gather


def test_world1_without_comm(tmp_path):
    res = _run(1, "none", 0, 13, str(tmp_path))
    want = _oracle(0, 13)
    assert {"polys": res[0]["polys"], "chal": res[0]["chal"], "blob_keccak": res[0]["blob_keccak"]} == want
    assert res[0]["collectives"] == 0


@pytest.mark.parametrize("nloc,gather", [(14, "0"), (14, "10"), (20, "10"), (13, "6")])
def test_rccl_data_path_forced_at_world1(tmp_path, nloc, gather):
    """ZK_FORCE_COLLECTIVES=1 runs a world-1 proof through the sharded code
    path over RCCL: every step's sums through ncclAllReduce + the publish
    kernel until the gather boundary, then the early gather as an in-place
    ncclAllGather (host.hpp gkr_prove_device) and k_interleave (gather 0:
    every step, then the one-element-per-table gather through the all-reduce)."""
    res = _run(1, "rccl", 0, nloc, str(tmp_path), {"ZK_FORCE_COLLECTIVES": "1", "ZK_GATHER_VARS": gather})
    want = _oracle(0, nloc)
    assert {"polys": res[0]["polys"], "chal": res[0]["chal"], "blob_keccak": res[0]["blob_keccak"]} == want
    assert res[0]["collectives"] == _collectives(nloc, int(gather))


@pytest.mark.parametrize("comm,world,nloc", [("host", 2, 10), ("rccl", 1, 12)])
def test_first_double_step_sharded(tmp_path, comm, world, nloc):
    """ZK_D0=1 (rounds 0 and 1 in one step over the inputs): its nine limb
    sums go through the same all-reduce as every other step."""
    env = {"ZK_D0": "1"}
    if comm == "rccl":
        env["ZK_FORCE_COLLECTIVES"] = "1"
    res = _run(world, comm, 0, nloc, str(tmp_path), env)
    want = _oracle(0, nloc + world.bit_length() - 1)
    for rank, r in enumerate(res):
        assert {"polys": r["polys"], "chal": r["chal"], "blob_keccak": r["blob_keccak"]} == want, f"rank {rank}"
        assert r["collectives"] == _collectives(nloc)


@pytest.mark.parametrize("world,nloc,field,gather", [(2, 16, 0, "0"), (2, 16, 2, "4"), (4, 13, 1, "6"), (2, 20, 0, "10"),
                                                     (2, 12, 0, "20")])
def test_early_gather_matches_single_process(tmp_path, world, nloc, field, gather):
    """ZK_GATHER_VARS: the ranks stop at the first step boundary leaving <= this
    many local rounds, fold by the pending challenges, gather every rank's
    tables with one all-reduce of a one-hot buffer, and finish the proof
    locally (0: run every local round, then gather one element per table).
    Every setting gives every rank the single-process oracle's proof."""
    res = _run(world, "host", field, nloc, str(tmp_path), {"ZK_GATHER_VARS": gather})
    want = _oracle(field, nloc + world.bit_length() - 1)
    for rank, r in enumerate(res):
        assert {"polys": r["polys"], "chal": r["chal"], "blob_keccak": r["blob_keccak"]} == want, f"rank {rank}"
        assert r["collectives"] == _collectives(nloc, int(gather)), f"rank {rank}"


# G = 8, the world size of the 8-GPU node, on this one card: 8 worker
# processes (host all-reduce over gloo; RCCL refuses ranks that share a
# device). Exercises the 8-way low-bit shard layout, the [8][4][2^T] gather
# buffer, the 8-way k_interleave and the last log2(8) = 3 rounds that every
# rank finishes locally (gather 0: the one-element-per-table gather).
@pytest.mark.parametrize("nloc,field,gather", [(10, 0, "10"), (14, 0, "0"), (13, 2, "10"), (12, 1, "6"), (14, 0, "10")])
def test_world8_host_comm_matches_single_process(tmp_path, nloc, field, gather):
    res = _run(8, "host", field, nloc, str(tmp_path), {"ZK_GATHER_VARS": gather})
    want = _oracle(field, nloc + 3)
    for rank, r in enumerate(res):
        assert {"polys": r["polys"], "chal": r["chal"], "blob_keccak": r["blob_keccak"]} == want, f"rank {rank}"
        assert r["collectives"] == _collectives(nloc, int(gather)), f"rank {rank}"


def test_config4_workload_8_ranks_matches_fixture(tmp_path):
    """BASELINE config 4's exact workload: the 26-variable seed-4 tables split
    over 8 ranks (23 local variables each: 8 x 1 GiB of tables on this one
    card, host all-reduce over gloo in place of RCCL). Every rank's proof must
    equal the committed full-size fixture (tests/golden/large.json
    bn254_fr_26_s4: round polynomials, challenges, blob digest), with the
    shipped collective schedule (per-step all-reduces, then the early gather)."""
    import json as _json

    fix = _json.load(open(os.path.join(ROOT, "tests", "golden", "large.json")))["bn254_fr_26_s4"]
    res = _run(8, "host", 0, 23, str(tmp_path), {"SEED": "4"})
    for rank, r in enumerate(res):
        assert r["polys"] == [[hex(int(c, 16)) for c in p] for p in fix["round_polys"]], f"rank {rank}"
        assert r["chal"] == [hex(int(c, 16)) for c in fix["challenges"]], f"rank {rank}"
        assert r["blob_keccak_claimed"] == fix["blob_keccak256"], f"rank {rank}"
        assert r["collectives"] == _collectives(23), f"rank {rank}"
        assert r["comm"] == {"kind": "host", "rank": rank, "count": 8}


# Peer reduction (zk_ctx_attach_peer_reduce): each step's publishing block
# writes its sums into every rank's IPC-mapped receive buffer and sums the
# world's itself. On this one card the ranks are processes sharing the device
# (host communicator for the handle exchange and the gather; steps launch after
# their challenges); at world 1 over RCCL (ZK_FORCE_COLLECTIVES=1) it runs the
# product schedule: pre-enqueued steps, no RCCL all-reduce or publish kernel.
# (gather <= 12 local variables: the early gather goes through the peers' gather
# buffers too, k_peer_gather; 14: it falls back to the communicator's)
@pytest.mark.parametrize("world,nloc,field,gather", [(2, 12, 0, "10"), (2, 16, 2, "0"), (4, 13, 1, "6"), (8, 14, 0, "10"),
                                                     (8, 10, 2, "0"), (2, 20, 0, "10"), (4, 0, 0, "10"), (2, 18, 0, "14"),
                                                     (4, 14, 0, "12")])
def test_peer_reduce_ranks_match_single_process(tmp_path, world, nloc, field, gather):
    res = _run(world, "host", field, nloc, str(tmp_path), {"PEER": "1", "ZK_GATHER_VARS": gather})
    want = _oracle(field, nloc + world.bit_length() - 1)
    for rank, r in enumerate(res):
        assert r["peer"] is True, f"rank {rank}"
        assert {"polys": r["polys"], "chal": r["chal"], "blob_keccak": r["blob_keccak"]} == want, f"rank {rank}"


@pytest.mark.parametrize("nloc,gather", [(14, "0"), (14, "10"), (20, "10"), (24, "10")])
def test_peer_reduce_forced_at_world1_rccl(tmp_path, nloc, gather):
    res = _run(1, "rccl", 0, nloc, str(tmp_path), {"PEER": "1", "ZK_FORCE_COLLECTIVES": "1", "ZK_GATHER_VARS": gather,
                                                    "SEED": "3" if nloc == 24 else "19"})
    assert res[0]["peer"] is True
    if nloc == 24:  # the headline workload: the committed fixture
        fix = json.load(open(os.path.join(ROOT, "tests", "golden", "large.json")))["bn254_fr_24_s3"]
        assert res[0]["chal"] == [hex(int(c, 16)) for c in fix["challenges"]]
        assert res[0]["blob_keccak_claimed"] == fix["blob_keccak256"]
        return
    want = _oracle(0, nloc)
    assert {"polys": res[0]["polys"], "chal": res[0]["chal"], "blob_keccak": res[0]["blob_keccak"]} == want
    assert res[0]["collectives"] == _collectives(nloc, int(gather))


def test_peer_reduce_config4_workload_8_ranks(tmp_path):
    """Config 4 (26 variables over 8 ranks) with the steps' sums through the
    peer buffers: every rank's proof equals the committed fixture."""
    fix = json.load(open(os.path.join(ROOT, "tests", "golden", "large.json")))["bn254_fr_26_s4"]
    res = _run(8, "host", 0, 23, str(tmp_path), {"SEED": "4", "PEER": "1"})
    for rank, r in enumerate(res):
        assert r["peer"] is True
        assert r["chal"] == [hex(int(c, 16)) for c in fix["challenges"]], f"rank {rank}"
        assert r["blob_keccak_claimed"] == fix["blob_keccak256"], f"rank {rank}"


@pytest.mark.parametrize("world,fail_rank", [(2, 1), (4, 0)])
def test_peer_attach_refused_on_every_rank_when_one_check_fails(tmp_path, world, fail_rank):
    """the attach-time check's outcome is agreed over the world. One
    rank's check is made to fail (ZK_PEER_CHECK_FAIL_RANK): EVERY rank's
    zk_ctx_attach_peer_reduce must then refuse (ZK_ECOMM), no rank may keep
    peer mode, and the proof that follows on the communicator must still be
    the oracle's on every rank (no rank waits in a peer kernel or the
    communicator for one that dropped out)."""
    res = _run(world, "host", 0, 12, str(tmp_path), {"PEER": "1", "PEER_MAY_FAIL": "1",
                                                    "ZK_PEER_CHECK_FAIL_RANK": str(fail_rank)})
    want = _oracle(0, 12 + world.bit_length() - 1)
    for rank, r in enumerate(res):
        assert r["peer"] is False and r["peer_refused"], f"rank {rank}"
        assert ("another rank" in r["peer_refused"]) == (rank != fail_rank), r["peer_refused"]
        assert {"polys": r["polys"], "chal": r["chal"], "blob_keccak": r["blob_keccak"]} == want, f"rank {rank}"
        assert r["collectives"] == _collectives(12)
