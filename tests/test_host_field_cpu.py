"""The hand-off's host field arithmetic (csrc/hfield.hpp) on the CPU: builds
tests/cpp/host_field_check.cpp with hipcc (host code only) and runs it."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_limb_conversion_fast_path_and_half(tmp_path):
    exe = str(tmp_path / "host_field_check")
    subprocess.run([HIPCC, "-O3", "-std=c++17", "-x", "c++",
                    "-I", os.path.join(ROOT, "zk-research-implementations_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "host_field_check.cpp"), "-o", exe],
                   check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "total mismatches 0" in r.stdout
