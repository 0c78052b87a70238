"""Sampler (HalogenRandom.hlsl): the oracle's restatement pinned against the reference's own table and
published constants; and the closed forms the HIP kernel uses proven equal to the literal table loop."""
import json
from pathlib import Path

import numpy as np

import hg_oracle

GOLD = Path(__file__).resolve().parent / "golden"


def test_sobol_table_matches_reference_text(built):
    """Oracle builds the table by the Joe–Kuo recurrence; the reference hard-codes it (HalogenRandom.hlsl:10-46)."""
    t = json.loads((GOLD / "sobol_table.json").read_text())["table"]
    L = hg_oracle.lib()
    for d in range(4):
        for b in range(32):
            assert L.hgo_sobol_table(d, b) == t[d][b], (d, b)


def _pcg_np(v):
    v = np.asarray(v, dtype=np.uint64)
    state = (v * np.uint64(747796405) + np.uint64(2891336453)) & np.uint64(0xFFFFFFFF)
    word = (((state >> ((state >> np.uint64(28)) + np.uint64(4))) ^ state) * np.uint64(277803737)) & np.uint64(0xFFFFFFFF)
    return ((word >> np.uint64(22)) ^ word).astype(np.uint32)


def test_pcg_hash_independent_restatement(built):
    L = hg_oracle.lib()
    xs = np.random.default_rng(1).integers(0, 2**32, 5000, dtype=np.uint64).astype(np.uint32)
    ref = _pcg_np(xs)
    got = np.array([L.hgo_pcg_hash(int(x)) for x in xs], dtype=np.uint32)
    assert np.array_equal(ref, got)
    assert L.hgo_pcg_hash(0) == int(_pcg_np([0])[0])


M32 = 0xFFFFFFFF


def brev(x):
    return int(f"{x:032b}"[::-1], 2)


def lk(x, seed):  # owen_scramble body, HalogenRandom.hlsl:154-158
    x ^= (x * 0x3D20ADEA) & M32
    x = (x + seed) & M32
    x = (x * ((seed >> 16) | 1)) & M32
    x ^= (x * 0x05526C56) & M32
    x ^= (x * 0x53A22864) & M32
    return x


def superset_xor(z):
    z ^= (z >> 1) & 0x55555555
    z ^= (z >> 2) & 0x33333333
    z ^= (z >> 4) & 0x0F0F0F0F
    z ^= (z >> 8) & 0x00FF00FF
    z ^= (z >> 16) & 0x0000FFFF
    return z


def test_closed_form_sobol_dims(built):
    """sobol1d(i,0) = brev(i); sobol1d(i,1) = brev(superset_xor(i)) — the kernel's loop-free forms."""
    L = hg_oracle.lib()
    rng = np.random.default_rng(2)
    for i in list(range(64)) + [int(v) for v in rng.integers(0, 2**32, 3000, dtype=np.uint64)]:
        assert L.hgo_sobol1d(i, 0) == brev(i)
        assert L.hgo_sobol1d(i, 1) == brev(superset_xor(i))


def test_closed_form_owen_sobol(built):
    """The kernel's get1/get2 (hg_trace.hip Sampler) equal u32_[2d_]owen_scrambled_sobol bit for bit."""
    import ctypes as C
    L = hg_oracle.lib()
    rng = np.random.default_rng(3)
    out = (C.c_uint32 * 2)()
    for _ in range(3000):
        idx, dim, seed = (int(v) for v in rng.integers(0, 2**32, 3, dtype=np.uint64))
        dim %= 4096
        s = seed ^ int(_pcg_np([dim])[0])
        one = brev(lk(idx, int(_pcg_np([s])[0])))
        assert L.hgo_u32_owen_scrambled_sobol(idx, dim, seed) == one
        sh = brev(lk(brev(idx), s))
        hc0 = s ^ ((0 + ((s << 6) & M32) + (s >> 2)) & M32)
        hc1 = s ^ ((1 + ((s << 6) & M32) + (s >> 2)) & M32)
        a = brev(lk(sh, hc0))
        b = brev(lk(superset_xor(sh), hc1))
        L.hgo_u32_2d_owen_scrambled_sobol(idx, dim, seed, out)
        assert (out[0], out[1]) == (a, b)


def test_blackman_harris_filter_shape(built):
    """The DebugSobol.compute idea as a KAT: 100k samples of index j, dim 0, seed 0 through the inverted
    Blackman–Harris CDF (DebugSobol.compute:31-40) — symmetric, within +-0.5, peaked at 0."""
    import ctypes as C
    L = hg_oracle.lib()
    out = (C.c_uint32 * 2)()
    xs = []
    for j in range(0, 100000, 7):
        L.hgo_u32_2d_owen_scrambled_sobol(j, 0, 0, out)
        xs.append(L.hgo_inverted_blackman_harris(out[0] / 4294967296.0))
    xs = np.array(xs)
    assert np.all(np.abs(xs) < 0.51)
    assert abs(xs.mean()) < 0.01
    h, _ = np.histogram(xs, bins=10, range=(-0.5, 0.5))
    assert h[4] + h[5] > 3 * (h[0] + h[9])
