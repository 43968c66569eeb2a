"""Shared test setup: import paths, the `gpu` marker, and fixtures."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cs265-lsm-tree_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: multi-second CPU work")


@pytest.fixture(scope="session")
def coracle():
    from bloom_oracle import COracle
    return COracle()


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(GOLDEN, "pins.json")) as f:
        return json.load(f)
