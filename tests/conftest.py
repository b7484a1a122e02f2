import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gym-lorenz_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


_GOLDEN_CACHE = {}


def golden(name):
    """Fixture arrays as a dict (an NpzFile re-decompresses on every item access)."""
    if name not in _GOLDEN_CACHE:
        with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
            _GOLDEN_CACHE[name] = {k: z[k] for k in z.files}
    return _GOLDEN_CACHE[name]


def bits_equal(a, b):
    """Bitwise equality, NaN-aware (any NaN matches any NaN)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return False
    an, bn = np.isnan(a), np.isnan(b)
    if not np.array_equal(an, bn):
        return False
    return np.array_equal(a[~an], b[~bn]) and np.array_equal(np.signbit(a[~an]), np.signbit(b[~bn]))


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.lib()
    return oracle
