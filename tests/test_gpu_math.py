"""GPU: the device restatement of Go's math (Cephes sin/cos/tan/atan/atan2/
asin), IEEE sqrt and division, and the S2 projections are bit-identical to the
CPU oracle's -- the precondition for bit-exact coverings."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def dev(op, x, y=None):
    from dss_amd import _lib
    ctx = _lib.context()
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.zeros_like(x)
    yp = np.ascontiguousarray(y, dtype=np.float64) if y is not None else None
    P = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    ctx.check(ctx.L.dssg_selftest_math(ctx.h, op, len(x), P(x), P(yp) if yp is not None else C.POINTER(C.c_double)(),
                                       P(out)))
    return out


def bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


@pytest.fixture(scope="module")
def xs():
    rng = np.random.default_rng(3)
    return np.concatenate([rng.uniform(-7, 7, 20000), rng.uniform(-1e-6, 1e-6, 2000), rng.uniform(-4e9, 4e9, 2000),
                           np.array([0.0, -0.0, 1e-300, np.pi, -np.pi, np.pi / 2, 3 * np.pi / 4])])


@pytest.mark.parametrize("op,name", [(0, "sin"), (1, "cos"), (2, "tan"), (3, "atan")])
def test_unary_go_math(oracle, xs, op, name):
    f = getattr(oracle.lib(), f"orc_go_{name}")
    ref = np.array([f(float(x)) for x in xs])
    assert np.array_equal(bits(dev(op, xs)), bits(ref))


def test_atan2_asin_sqrt_div(oracle, xs):
    rng = np.random.default_rng(4)
    ys = rng.uniform(-7, 7, len(xs))
    ref = np.array([oracle.lib().orc_go_atan2(float(a), float(b)) for a, b in zip(xs, ys)])
    assert np.array_equal(bits(dev(4, xs, ys)), bits(ref))
    u = rng.uniform(-1, 1, 5000)
    ref = np.array([oracle.lib().orc_go_asin(float(a)) for a in u])
    assert np.array_equal(bits(dev(5, u)), bits(ref))
    p = np.abs(xs)
    assert np.array_equal(bits(dev(6, p)), bits(np.sqrt(p)))
    assert np.array_equal(bits(dev(7, xs, ys)), bits(xs / ys))


def test_point_from_degrees(oracle):
    rng = np.random.default_rng(5)
    la = rng.uniform(-90, 90, 5000)
    lg = rng.uniform(-180, 180, 5000)
    ref = np.array([oracle.point_from_degrees(a, b)[0] for a, b in zip(la, lg)])
    assert np.array_equal(bits(dev(10, la, lg)), bits(ref))
