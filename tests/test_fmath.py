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


def test_sincos_fused_is_bit_identical(built):
    """hg_sincosf (the device kernels' call) returns exactly (hg_sinf(x), hg_cosf(x)): random bit patterns over the
    whole float range, the kernels' argument ranges, octant boundaries and the special values."""
    rng = np.random.default_rng(11)
    x = np.concatenate([
        rng.integers(0, 2**32, 400000, dtype=np.uint64).astype(np.uint32).view(np.float32),
        rng.uniform(0.0, 2 * np.pi, 200000).astype(np.float32),       # theta = u * 2 pi
        rng.uniform(0.0, np.pi, 200000).astype(np.float32),           # phi = acos(2u - 1)
        (np.arange(-64, 65, dtype=np.float32) * np.float32(np.pi / 4)),
        np.nextafter(np.arange(-64, 65, dtype=np.float32) * np.float32(np.pi / 4), np.float32(np.inf)),
        np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-30, -1e-30, 3e38, -3e38], np.float32)])
    for fn_fused, fn_ref in ((9, 0), (10, 1)):
        a, b = _eval(fn_fused, x), _eval(fn_ref, x)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (fn_fused, x[a.view(np.uint32) != b.view(np.uint32)][:8])


def test_acos_fused_exhaustive(built):
    """hg_acosf_fused (the device kernels' call) equals hg_acosf bitwise on every float in [-1, 1] (~2.1e9 inputs,
    about 12 s); hg_sincosf was checked the same way over [0, 2*pi] (0 mismatches, 130 s, not rerun here)."""
    L = hg_oracle.lib()
    L.hgo_fused_mismatches.restype = C.c_int64
    L.hgo_fused_mismatches.argtypes = [C.c_int32, C.c_uint32, C.c_uint32]
    one = int(np.float32(1.0).view(np.uint32))
    assert L.hgo_fused_mismatches(1, 0, one) == 0
    assert L.hgo_fused_mismatches(1, 0x80000000, 0x80000000 | one) == 0
