"""Multi-rank path on CPU (gloo, world_size 2 and 4), modelling the SHIPPED
collective schedule.

Each rank holds its low-index-bit shard of the four GKR tables (local m <->
global m * world + rank) and runs the step schedule the device code runs
(host.hpp gkr_phase / gkr_prove_device, tests/gkr_schedule.py):

* each step covers 1, 2 or 3 rounds and exchanges exactly what the device
  step publishes: round 0 alone — e0, e1, e2; a single round — e0, e2; a
  two-round step — the grid-point product sums V_ab (a, b in {0, 1, 2}; eight
  categories, nine in the first step: V11 gives round 0's e1); a three-round
  step — the 27 moment sums (per axis X0Y0, X1Y1, X0Y1 + X1Y0) of the
  k_gkr_d0t / k_gkr_t33 tiles;
* ONE limb-split u64 all-reduce per step (zk_amd.dist.TorchAllreduce, the host
  communicator the library calls back into), then every rank derives the
  step's rounds with the host's formulas (three_rounds / two_rounds) from an
  identical transcript;
* at the first step boundary leaving <= ZK_GATHER_VARS local rounds every rank
  folds by the pending challenges, the folded tables of all ranks are gathered
  in one collective (the host communicator's one-hot all-reduce; RCCL: an
  in-place ncclAllGather), interleaved to the global layout, and every rank
  finishes the proof locally; without such a boundary every step runs across
  ranks and one element per table is gathered at the end.

Every rank's proof must equal the single-process oracle's over the full
tables, and the number of collectives must equal the library's schedule.
Per-shard arithmetic is plain Python over the oracle's field (test
infrastructure).
"""
from __future__ import annotations

import json
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 17


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _corner(tab, idx_bits, nb, q):
    """Element of a table at corner idx_bits (nb leading variables) of block q."""
    L = len(tab)
    return tab[idx_bits * (L >> nb) + q]


def _grid(p, tab, nb, q, pt):
    """The table's multilinear extension in its nb leading variables at grid
    point pt (coordinates in {0, 1, 2}), block q."""
    vals = {}
    for c in range(1 << nb):
        vals[c] = _corner(tab, c, nb, q)
    # extend one axis at a time: X(2) = 2 X(1) - X(0)
    for axis in range(nb):
        sh = nb - 1 - axis
        t = pt[axis]
        nxt = {}
        for c, v in vals.items():
            if (c >> sh) & 1:
                continue
            x0, x1 = v, vals[c | (1 << sh)]
            nxt[c] = x0 if t == 0 else x1 if t == 1 else (2 * x1 - x0) % p
        vals = nxt
    return vals[0]


def _step_sums(p, tabs, nb, first):
    """What one device step publishes, as field values (mod p)."""
    A, S, M, P = tabs
    nq = len(A) >> nb
    if nb == 1:
        pts = [(0,), (1,), (2,)] if first else [(0,), (2,)]
    elif nb == 2:
        # categories (kernels.hpp): 0 V00, 1 V22, 2 V01, 3 V02, 4 V10, 5 V20, 6 V21, 7 V12 (+ 8 V11 first)
        pts = [(0, 0), (2, 2), (0, 1), (0, 2), (1, 0), (2, 0), (2, 1), (1, 2)] + ([(1, 1)] if first else [])
    else:
        pts = None
    if pts is not None:
        out = []
        for pt in pts:
            acc = 0
            for q in range(nq):
                acc += _grid(p, A, nb, q, pt) * _grid(p, S, nb, q, pt) + _grid(p, M, nb, q, pt) * _grid(p, P, nb, q, pt)
            out.append(acc % p)
        return out
    # three rounds: 27 moment tiles, id 9 alpha + 3 beta + gamma; per axis
    # moment 0 = X0 Y0, 1 = X1 Y1, 2 = X0 Y1 + X1 Y0 over the octant's corners
    sel = {0: [(0, 0)], 1: [(1, 1)], 2: [(0, 1), (1, 0)]}
    T = [0] * 27
    for q in range(nq):
        cx = [[_corner(X, c, 3, q) for c in range(8)] for X in (A, M)]
        cy = [[_corner(Y, c, 3, q) for c in range(8)] for Y in (S, P)]
        for a in range(3):
            for b in range(3):
                for g in range(3):
                    acc = 0
                    for ua, va in sel[a]:
                        for ub, vb in sel[b]:
                            for ug, vg in sel[g]:
                                u, v = 4 * ua + 2 * ub + ug, 4 * va + 2 * vb + vg
                                acc += cx[0][u] * cy[0][v] + cx[1][u] * cy[1][v]
                    T[9 * a + 3 * b + g] += acc
    return [t % p for t in T]


class _Prover:
    """The host side of gkr_phase: transcript, claim, the step formulas."""

    def __init__(self, field):
        import pyoracle as po

        self.po, self.p = po, po.MODULI[field]
        self.tr = po.Transcript(field)
        self.polys, self.chal, self.claim = [], [], 0

    def one_round(self, e0, e1, e2):
        po, p = self.po, self.p
        c = po.interpolate(p, [0, 1, 2], [e0 % p, e1 % p, e2 % p])
        self.tr.append(po.fq_vec_to_bytes(c))
        r = self.tr.get_random_challenge()
        self.polys.append(c)
        self.chal.append(r)
        self.claim = po.uni_evaluate(p, c, r)
        return r

    def step(self, v, nb, first):
        p = self.p
        if nb == 1:
            if first:
                self.one_round(*v)
            else:
                self.one_round(v[0], self.claim - v[0], v[1])
        elif nb == 2:  # host.hpp two_rounds
            e0 = v[0] + v[2]
            e1 = v[4] + v[8] if first else self.claim - e0
            r = self.one_round(e0, e1, v[5] + v[6])
            inv2 = pow(2, -1, p)
            L0, L1, L2 = (r - 1) * (r - 2) * inv2, -r * (r - 2), r * (r - 1) * inv2
            f0 = (L0 * v[0] + L1 * v[4] + L2 * v[5]) % p
            f2 = (L0 * v[3] + L1 * v[7] + L2 * v[1]) % p
            self.one_round(f0, self.claim - f0, f2)
        else:  # host.hpp three_rounds: X(t) Y(t) = (1-t)^2 m0 + t^2 m1 + t(1-t) ms
            T = v
            at2 = lambda m0, m1, ms: m0 + 4 * m1 - 2 * ms  # noqa: E731
            wts = lambda t: [(1 - t) * (1 - t) % p, t * t % p, t * (1 - t) % p]  # noqa: E731
            U = [T[9 * a] + T[9 * a + 1] + T[9 * a + 3] + T[9 * a + 4] for a in range(3)]
            ra = self.one_round(U[0], U[1] if first else self.claim - U[0], at2(*U))
            wa = wts(ra)
            V = [sum(wa[a] * (T[9 * a + 3 * b] + T[9 * a + 3 * b + 1]) for a in range(3)) % p for b in range(3)]
            rb = self.one_round(V[0], self.claim - V[0], at2(*V))
            wb = wts(rb)
            Z = [sum(wa[a] * sum(wb[b] * T[9 * a + 3 * b + g] for b in range(3)) for a in range(3)) % p
                 for g in range(3)]
            self.one_round(Z[0], self.claim - Z[0], at2(*Z))

    def local_rounds(self, tabs, nv):
        """Rounds run by every rank alone after the gather (same values as any
        step grouping: the sums are exact)."""
        po, p = self.po, self.p
        for i in range(nv):
            self.step(_step_sums(p, tabs, 1, True), 1, True)
            tabs = [po.partial_evaluate(p, tb, 0, self.chal[-1]) for tb in tabs]
        return tabs


def _worker(rank: int, world: int, port: int, field: int, n_local: int, gather_vars: int, out_dir: str) -> None:
    for p in (os.path.join(ROOT, "zk-research-implementations_amd"), os.path.join(ROOT, "oracle"),
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import coracle as co
    import gkr_schedule
    import pyoracle as po
    from zk_amd.dist import TorchAllreduce, limb_join, limb_split, shard_layout

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    ar = TorchAllreduce()
    ncoll = 0

    def allreduce(vals):
        nonlocal ncoll
        vec = limb_split(vals)
        ar(vec)
        ncoll += 1
        return limb_join(vec, p)

    p = po.MODULI[field]
    lg = world.bit_length() - 1
    i0, stride = shard_layout(rank, world)
    n = n_local + lg
    cur = [co.from_limbs(co.synth(field, SEED, t, 0, 1 << n))[i0::stride] for t in range(4)]
    pv = _Prover(field)
    bnds = gkr_schedule.bounds(n_local)
    gs = gkr_schedule.gather_step(n_local, gather_vars)
    start, pending = 0, []
    stopped = None
    for s, e in enumerate(bnds):
        for r in pending:  # the step folds by the previous step's challenges first
            cur = [po.partial_evaluate(p, tb, 0, r) for tb in cur]
        nb = e - start
        first = start == 0
        pv.step(allreduce(_step_sums(p, cur, nb, first)), nb, first)
        pending = pv.chal[start:e]
        start = e
        if gs is not None and s == gs:
            stopped = e
            break
    for r in pending:  # fold by the pending challenges (the last one included)
        cur = [po.partial_evaluate(p, tb, 0, r) for tb in cur]
    T = n_local - (stopped if stopped is not None else n_local)
    if lg or stopped is not None:
        # one collective gathers every rank's 4 x 2^T folded elements (one-hot slots)
        vals = [0] * (world * 4 << T)
        for t in range(4):
            vals[(rank * 4 + t) << T: (rank * 4 + t + 1) << T] = cur[t]
        g = allreduce(vals)
        # global table t: index m * world + rank' = rank' slot's element m
        glob = [[g[((k % world) * 4 + t << T) + k // world] for k in range(world << T)] for t in range(4)]
        pv.local_rounds(glob, T + lg)
    res = {"polys": [[hex(x) for x in c] for c in pv.polys], "chal": [hex(x) for x in pv.chal],
           "collectives": ncoll}
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as fh:
        json.dump(res, fh)
    dist.destroy_process_group()


# (world, n_local, gather): three-round steps (d0t, t33), the dm3 step, doubles
# and the early gather at 10 / 6; the small-n schedules (round 0 + singles,
# rounds 0-1) with the final one-element gather; an empty local cube
@pytest.mark.parametrize("world,n_local,gather", [(2, 13, 10), (4, 16, 6), (2, 8, 0), (4, 9, 10), (2, 7, 3), (2, 0, 10)])
def test_shipped_schedule_matches_single_process(tmp_path, world, n_local, gather):
    import torch.multiprocessing as mp

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle as co
    import gkr_schedule

    field = 0
    mp.spawn(_worker, args=(world, _free_port(), field, n_local, gather, str(tmp_path)), nprocs=world, join=True)
    n = n_local + world.bit_length() - 1
    tabs = [co.synth(field, SEED, t, 0, 1 << n) for t in range(4)]
    polys, chal = co.gkr_prove(field, tabs, co.Transcript())
    want = {"polys": [[hex(x) for x in c] for c in polys], "chal": [hex(x) for x in chal],
            "collectives": gkr_schedule.collectives(n_local, gather) if world > 1 else 0}
    for rank in range(world):
        with open(tmp_path / f"rank{rank}.json") as fh:
            assert json.load(fh) == want, f"rank {rank}"


def test_schedule_shapes():
    """The schedule helper against hand-derived schedules (host.hpp gkr_phase)."""
    import gkr_schedule as gs

    assert gs.bounds(24) == [3, 6, 9, 12, 14, 16, 18, 20, 22, 24]  # d0t, t33 x3, dm3, doubles
    assert gs.bounds(23) == [3, 6, 9, 11, 13, 15, 17, 19, 21, 23]  # d0t, t33 x2, dm3 at an odd level, doubles
    assert gs.bounds(16) == [3, 6, 8, 10, 12, 14, 16]
    assert gs.bounds(9) == [1, 2, 3, 5, 7, 9]  # round 0, two single rounds, doubles
    assert gs.bounds(8) == [2, 4, 6, 8]  # rounds 0-1, doubles
    # config 4 on 8 ranks (23 local variables): five steps across ranks, the
    # gather at 10 local rounds left, then every rank alone
    assert gs.gather_step(23) == 4 and gs.bounds(23)[4] == 13 and gs.collectives(23) == 6
    assert gs.collectives(8, 0) == 5  # no gather boundary: every step + the final one-element gather
