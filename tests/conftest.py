import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "trapped-modes-ltg_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs the engine's kernels")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return load


def border_ring(shape, width=1):
    m = np.zeros(shape, bool)
    m[:width] = m[-width:] = True
    m[:, :width] = m[:, -width:] = True
    return m


def same_up_to_constant(a, b):
    """k-fields equal up to one global integer (the unwrap's anchor)."""
    d = np.asarray(a, np.int64) - np.asarray(b, np.int64)
    return d - d.flat[0]
