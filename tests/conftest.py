"""Shared test setup.

`-m "not gpu"` (CPU, here): oracle vs golden vectors and the reference's KATs,
host logic of the library (transcript, serialisation, gkr_verify), that the
C-ABI library loads and exports every declared symbol, and the multi-rank
exchange path over gloo.
`-m gpu` (MI355X): parity of the HIP path with the oracle through the C ABI.
"""
from __future__ import annotations

import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "zk-research-implementations_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity through the C ABI")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def ctx():
    """One device context for the whole GPU session (tests run in one process)."""
    import zk_amd

    return zk_amd.default_context(0)


def h2i(s: str) -> int:
    return int(s, 16)
