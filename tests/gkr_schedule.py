"""The step schedule of a sharded GKR sum-check (test helper, not a test
module): which rounds each device step covers and how many collectives a
sharded proof makes, as host.hpp `gkr_phase` / `gkr_prove_device` build them.
Shared by tests/test_gpu_sharded.py (checks the library's collective count)
and tests/test_dist_cpu.py (runs the same schedule over gloo on the CPU)."""
from __future__ import annotations


def bounds(nloc: int, d0: bool = True) -> list[int]:
    """End round of each step of a sharded phase (no persistent steps across
    ranks), as host.hpp gkr_phase builds the schedule: n >= 11 — the input
    pass over rounds 0-2, triple steps, one two-round step (dm3), double steps;
    smaller — round 0 (+ one or two single rounds) or rounds 0-1, then doubles."""
    b: list[int] = []
    if nloc == 0:
        return b
    if d0 and nloc >= 11:
        nt, k = -1, 0
        while 3 + 3 * k + 8 <= nloc:
            r = nloc - 3 - 3 * k
            if r % 2 == 0 and (r >= 12 or nt < 0):
                nt = k
            k += 1
        b = [3 + 3 * k for k in range(nt + 1)] + [5 + 3 * nt]
        i = 5 + 3 * nt
    elif d0 and nloc >= 2 and nloc % 2 == 0:
        b, i = [2], 2
    else:
        b, i = [1], 1
        if nloc >= 2:
            i += 1
            b.append(i)
        if nloc >= 3 and (nloc - 2) % 2 == 1:
            i += 1
            b.append(i)
    while i + 1 < nloc:
        i += 2
        b.append(i)
    return b


def gather_step(nloc: int, gather_vars: int = 10, d0: bool = True) -> int | None:
    """Index of the step after which the ranks gather their folded tables
    (the first step boundary leaving <= gather_vars local rounds), or None:
    then every step runs across ranks and one element per table is gathered
    at the end."""
    if gather_vars > 0:
        for s, e in enumerate(bounds(nloc, d0)):
            if e < nloc and nloc - e <= gather_vars:
                return s
    return None


def collectives(nloc: int, gather_vars: int = 10, d0: bool = True) -> int:
    """All-reduces of a sharded proof (world > 1): one per step until the
    gather boundary, then ONE gather of the folded tables (host.hpp
    gkr_prove_device); every later round runs locally on every rank. Without
    such a boundary: every step + the final gather of one element per table."""
    s = gather_step(nloc, gather_vars, d0)
    return s + 2 if s is not None else len(bounds(nloc, d0)) + 1
