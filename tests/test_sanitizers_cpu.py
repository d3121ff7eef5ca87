"""Host sanitizers (VERDICT r2 "next" 8): ASan + UBSan builds of
(1) the C oracle with tests/native/oracle_asan_check.c and (2) the product
library's host side (`-Xarch_host -fsanitize=...`: device code is never
sanitised) with tests/native/host_asan_check.cpp, which drives every C-ABI
entry point that does no device work on valid and hostile inputs (transcript
state images, truncated and bit-flipped proof blobs, random proofs through
gkr_verify and circuit verify, pairings, zk_ctx_create without a GPU). Any
sanitizer report aborts the checker (-fno-sanitize-recover=all)."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

from conftest import ROOT

PKG = os.path.join(ROOT, "zk-research-implementations_amd")
ORACLE = os.path.join(ROOT, "oracle")


def _gpu_present() -> bool:
    return os.path.exists("/dev/kfd")


def _run(exe: str, **env) -> str:
    e = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1", **env)
    r = subprocess.run([exe], capture_output=True, text=True, env=e, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return r.stdout


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no C compiler")
def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", ORACLE, "asan"], check=True, timeout=600)
    assert "oracle_asan_check ok" in _run(os.path.join(ORACLE, "build", "oracle_asan_check"), OMP_NUM_THREADS="4")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not present")
@pytest.mark.skipif(_gpu_present(), reason="the checker expects zk_ctx_create to fail without a GPU")
def test_library_host_side_under_asan_ubsan():
    # __graft_entry__.build() builds this target too; make is a no-op when it is up to date
    jobs = os.environ.get("MAX_JOBS", "8")
    subprocess.run(["make", "-s", "-j", jobs, "-C", PKG, "asan"], check=True, timeout=1800)
    assert "host_asan_check ok" in _run(os.path.join(PKG, "build", "asan", "host_asan_check"))
