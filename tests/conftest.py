import os
import sys

import pytest
# torch first, as in bench.py and in a full collection (test_dist_gloo imports it): the engine
# library then binds to the HIP runtime torch has loaded.  A test that imports torch only after
# the engine library initialised HIP (the protocol-mirror test spawns gloo ranks) otherwise
# brings torch's ROCm libraries in on top of another runtime, and the process aborts at exit
# ("double free or corruption", round 5).
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "barnes-hut-n-body_amd")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


def bits_equal(a, b):
    import numpy as np
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64))


@pytest.fixture(scope="session")
def engine_lib():
    import bh_amd
    return bh_amd.load_library()
