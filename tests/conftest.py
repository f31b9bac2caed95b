import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return np.load(os.path.join(GOLDEN, "golden.npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def gpu_lib():
    """libga_amd.so with comex initialised on cuda:0 (GPU tests only)."""
    import ga_amd
    L = ga_amd.lib()
    if L.gaamd_device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    assert ga_amd.comex_init() == 0
    yield L
    L.comex_finalize()
