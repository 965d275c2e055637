"""Test configuration: package path, the `gpu` marker, shared fixtures.

`-m "not gpu"` (CPU, this container): oracle vs golden vectors, host logic, C-ABI exports.
`-m gpu` (MI355X box): parity of the HIP path against the oracle and the golden vectors.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "radar-point-cloud-tracking_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU and librpt.so")
    _heartbeat()


def _heartbeat():
    """RPT_HEARTBEAT=<file>: append the running test's id every 30 s (long full-size tests keep
    a watcher that judges liveness by output -- gpurun's 3-minute rule -- informed; per-test
    hangs are still ended by pytest-timeout)."""
    import os
    import threading
    import time

    path = os.environ.get("RPT_HEARTBEAT")
    if not path:
        return

    def beat():
        while True:
            time.sleep(30)
            try:
                with open(path, "a") as fh:
                    fh.write(f"{time.strftime('%H:%M:%S')} "
                             f"{os.environ.get('PYTEST_CURRENT_TEST', '-')}\n")
            except OSError:
                pass

    threading.Thread(target=beat, daemon=True).start()


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(GOLDEN / name, allow_pickle=False)
    return load


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test run without a visible GPU")
    from rpt import _abi

    _abi.load()
    return torch.device("cuda", 0)
