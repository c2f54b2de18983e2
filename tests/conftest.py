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

# torch (used by some GPU tests for device buffers) ships its own libamdhip64.so.7;
# loaded first, it is the one HIP runtime the engine library binds to as well (same
# soname).  Loaded after the engine's /opt/rocm runtime it would be a second runtime
# in the process, which finds no devices.  INTEGRATION.md §3.
try:
    import torch  # noqa: F401
except ImportError:
    pass


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


def spectrum_images(golden):
    """(fixture, {name: float32 image}) of tests/golden/spectrum.npz (make_golden.py
    spectrum_images): the c2 board flat and rotated, the example references, stored
    integer-valued images of other shapes."""
    from bench_data import checkerboard
    g = golden("spectrum")
    imgs = {"board_flat": checkerboard(1024), "board_rot5": checkerboard(1024, 5.0),
            "reference_2": golden("real_pair")["ref_u8"].astype(np.float32),
            "reference_df": golden("real_df")["ref_u16"].astype(np.float32)}
    for name in g["names"]:
        name = str(name)
        if name.startswith("rand_"):
            imgs[name] = g[name + "_u16"].astype(np.float32) * np.float32(0.37)
    return g, imgs
