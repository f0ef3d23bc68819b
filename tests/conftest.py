import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device and libdss_amd.so")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def golden_covering():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "covering.npz"), allow_pickle=False))


@pytest.fixture(scope="session")
def golden_search():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "search.npz"), allow_pickle=False))


@pytest.fixture(params=["units", "units_dense", "small"])
def join_path(request):
    """Run a search test through every join of the shared context: "units"
    (the tiled band join, one 64-posting tile per unit: k_join in its sparse
    shape, 7 workgroups per CU with 640-pair stages; small_search = 0),
    "units_dense" (the same join in its dense shape, 6 x 1024) and "small"
    (the one-launch small-batch join, k_small_join, forced for every
    batch)."""
    from dss_amd import _lib
    ctx = _lib.context(0)
    ctx.set_tuning("small_search", 1 << 24 if request.param == "small" else 0)
    ctx.set_tuning("join_shape", 2 if request.param == "units_dense" else 1)
    try:
        yield request.param
    finally:
        ctx.set_tuning("small_search", 4096)
        ctx.set_tuning("join_shape", 0)
