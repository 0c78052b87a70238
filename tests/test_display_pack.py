"""The display formats of hg_readback_begin_format (csrc/hg_pack.h, include/halogen_abi.h), on the host: the library's
hg_pack_display against independent restatements.  R11G11B10F is what the reference displays: its accumulation target
is blitted into the URP HDR camera target (HalogenRenderPass.cs:345), R11G11B10 per URP-HighFidelity.asset:26-27.
Parity with D3D's own float -> R11G11B10 converter is UNPINNED (no D3D here); the rules are ours and documented: round
to nearest even, overflow to +Inf, negatives and NaN to 0.  The device packing is compared with this host packing in
tests/test_gpu_display.py.  No GPU needed."""
import math

import numpy as np
import pytest

from halogen import abi


def ref_ufloat(x: float, mbits: int) -> int:
    """Unsigned float, 5-bit exponent (bias 15), mbits mantissa bits, by exact float64 arithmetic."""
    if math.isnan(x) or x <= 0.0:
        return 0
    inf = 31 << mbits
    if math.isinf(x):
        return inf
    m, e = math.frexp(x)  # x = m 2^e, m in [0.5, 1)
    E = e - 1
    normal = E >= -14
    unit = math.ldexp(1.0, (E - mbits) if normal else (-14 - mbits))
    n = round(x / unit)  # exact quotient (power-of-2 unit); Python rounds half to even
    field = (((E + 15) << mbits) + n - (1 << mbits)) if normal else n
    return min(field, inf)


def ref_r11g11b10(r, g, b) -> int:
    return ref_ufloat(r, 6) | (ref_ufloat(g, 6) << 11) | (ref_ufloat(b, 5) << 22)


def special_values():
    f = np.float32
    vals = [0.0, -0.0, 1.0, -1.0, 0.5, 2.0, 65024.0, 65535.0, 65536.0, 64512.0, 64513.0, 66000.0, 1e30, -1e30,
            float("inf"), -float("inf"), float("nan"), -float("nan"),
            2.0 ** -14, 2.0 ** -15, 2.0 ** -20, 2.0 ** -21, 2.0 ** -19, 3 * 2.0 ** -21, 2.0 ** -25, 1e-40, -1e-40,
            np.nextafter(f(2.0 ** -14), f(0)), np.nextafter(f(65024.0), f(1e9)), 1.0 + 2.0 ** -7, 1.0 + 3 * 2.0 ** -7,
            1.0 + 2.0 ** -6, 1.0 + 2.0 ** -6 + 2.0 ** -7, 0.18, 0.735, 3.14159]
    # halfway cases of every mantissa width used: 1 + k 2^-m + 2^-(m+1)
    for m in (5, 6, 10):
        for k in (0, 1, 2, 3):
            vals.append(1.0 + k * 2.0 ** -m + 2.0 ** -(m + 1))
            vals.append(2.0 ** -16 * (1.0 + k * 2.0 ** -m + 2.0 ** -(m + 1)))
    return np.array(vals, dtype=np.float32)


def sample_values(n=20000, seed=11):
    rng = np.random.default_rng(seed)
    bits = rng.integers(0, 2 ** 32, size=n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    logu = (10.0 ** rng.uniform(-9, 5.5, size=n)).astype(np.float32)
    return np.concatenate([special_values(), bits, logu, -logu[:100]])


def as_pixels(v):
    n = (len(v) + 3) // 4 * 4
    v = np.concatenate([v, np.zeros(n - len(v), np.float32)])
    return v.reshape(-1, 4)


def test_r11g11b10_matches_restatement(built):
    px = as_pixels(sample_values())
    got = abi.pack_display(px, abi.HG_DISPLAY_R11G11B10F)
    want = np.array([ref_r11g11b10(float(p[0]), float(p[1]), float(p[2])) for p in px], np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(px[i].tolist(), hex(int(got[i])), hex(int(want[i]))) for i in bad[:5]]


def test_r11g11b10_fields():
    """Known encodings: 1.0 = exponent 15, mantissa 0; the largest finite values; Inf; bit positions."""
    assert ref_ufloat(1.0, 6) == 15 << 6 and ref_ufloat(1.0, 5) == 15 << 5
    assert ref_ufloat(65024.0, 6) == (30 << 6) | 63 and ref_ufloat(64512.0, 5) == (30 << 5) | 31
    assert ref_ufloat(65536.0, 6) == 31 << 6 and ref_ufloat(float("inf"), 5) == 31 << 5
    assert ref_ufloat(2.0 ** -20, 6) == 1 and ref_ufloat(2.0 ** -21, 6) == 0  # smallest denormal; its half ties to 0
    assert ref_r11g11b10(1.0, 0.0, 0.0) == 15 << 6
    assert ref_r11g11b10(0.0, 1.0, 0.0) == (15 << 6) << 11
    assert ref_r11g11b10(0.0, 0.0, 1.0) == (15 << 5) << 22


def test_rgba16f_matches_numpy(built):
    px = as_pixels(sample_values())
    got = abi.pack_display(px, abi.HG_DISPLAY_RGBA16F).view(np.uint16)
    with np.errstate(over="ignore", invalid="ignore"):
        want = px.astype(np.float16).view(np.uint16).copy()
    nan = np.isnan(px)
    want[nan] = 0x7E00  # our NaN rule: the quiet NaN 0x7E00 (numpy keeps sign and payload bits)
    bad = np.argwhere(got != want)
    assert bad.size == 0, [(float(px[tuple(i)]), hex(int(got[tuple(i)])), hex(int(want[tuple(i)]))) for i in bad[:5]]


def test_rgba32f_is_identity(built):
    px = as_pixels(sample_values(2000))
    got = abi.pack_display(px, abi.HG_DISPLAY_RGBA32F)
    assert np.array_equal(got.view(np.uint32), px.view(np.uint32))


def test_bad_format_is_refused(built):
    with pytest.raises(ValueError):
        abi.pack_display(np.zeros((2, 4), np.float32), 7)
