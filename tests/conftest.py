"""Test configuration.  GPU tests are marked `gpu`; everything else runs on CPU.

Both native libraries are built in-tree on demand: libpebble_amd.so (hipcc,
gfx950; host-side entry points such as the writer work without a GPU) and the
oracle's liboracle.so (gcc).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session", autouse=True)
def _native_libs():
    import oracle
    from pebble_amd import build as B
    if not os.path.exists(B.OUT):
        B.build()
    oracle.build()
    yield


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(TESTS, "golden", "rowblk_golden.json")) as f:
        return json.load(f)


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
