"""The host C++ of librpt under AddressSanitizer + UndefinedBehaviorSanitizer:
tools/asan/Makefile builds the host-only units (csv.cpp -- the radar CSV parser fed untrusted
files like 4_temporal_object_tracker.py:191-198 --, tracker.cpp, shard_host.cpp, errors.cpp)
with -fsanitize=address,undefined into librpt_host_asan.so and runs the host tests (CSV ingest
incl. malformed files, the shard host stage, the tracker / LSAP / cluster order) through an
interpreter with the sanitizer runtimes linked first.  Any report aborts the run."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.timeout(900)
def test_host_units_clean_under_asan_ubsan():
    if not shutil.which("g++") or not shutil.which("python3-config"):
        pytest.skip("no host toolchain for the sanitizer build")
    r = subprocess.run(["make", "-s", "-C", str(ROOT / "tools" / "asan"), "check"],
                       capture_output=True, text=True, timeout=880)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-6000:]
    assert " passed" in out, out[-3000:]
