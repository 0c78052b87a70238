"""include/hg_fmath.h — the arithmetic spec shared by kernel and oracle — against libm (float64)."""
import ctypes as C

import numpy as np
import pytest

import hg_oracle

FNS = {"sin": (0, (0.0, 7.0), np.sin, 2.0), "cos": (1, (0.0, 7.0), np.cos, 2.0),
       "acos": (2, (-1.0, 1.0), np.arccos, 2.0), "tan": (3, (0.0, 1.5), np.tan, 3.0),
       "log": (4, (1e-3, 600.0), np.log, 1.5), "exp": (5, (-80.0, 5.0), np.exp, 1.5),
       "asin": (8, (-1.0, 1.0), np.arcsin, 3.0)}


def _eval(fn, x):
    L = hg_oracle.lib()
    L.hgo_fmath.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_int64]
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    L.hgo_fmath(fn, x.ctypes.data, y.ctypes.data, x.size)
    return y


@pytest.mark.parametrize("name", sorted(FNS))
def test_accuracy_ulp(built, name):
    fn, dom, ref, max_ulp = FNS[name]
    x = np.random.default_rng(7).uniform(*dom, size=100000).astype(np.float32)
    y = _eval(fn, x).astype(np.float64)
    r = ref(x.astype(np.float64))
    ulp = np.abs(y - r) / np.spacing(np.abs(r.astype(np.float32))).astype(np.float64)
    assert ulp.max() <= max_ulp, (name, ulp.max())


def test_special_values(built):
    nan = np.float32(np.nan)
    assert np.isnan(_eval(0, [nan])[0]) and np.isnan(_eval(4, [-1.0])[0])
    assert _eval(4, [0.0])[0] == -np.inf
    assert _eval(5, [-200.0])[0] == 0.0 and _eval(5, [100.0])[0] == np.inf
    assert _eval(2, [1.0])[0] == 0.0


def test_round_half_even(built):
    x = np.array([0.5, 1.5, 2.5, -0.5, -1.5, 2.4999998, 3.5000002, 8388609.0], np.float32)
    assert np.array_equal(_eval(6, x), np.rint(x))


def test_rnorm_is_ieee(built):
    x = np.random.default_rng(9).uniform(1e-6, 1e6, 10000).astype(np.float32)
    expect = (np.float32(1.0) / np.sqrt(x)).astype(np.float32)
    assert np.array_equal(_eval(7, x), expect)
