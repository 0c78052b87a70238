"""Synthetic HDR environment cubemap (the reference's resting_place_4k.exr is a missing blob,
.MISSING_LARGE_BLOBS:1-3; its import settings — cubemap, specular-convolved mips, HDR — are in
Assets/Environments/resting_place_4k.exr.meta:30-35,62).

Layout matches hg_upload_cubemap: RGBA32F, [mip][face][y][x][4], faces +X,-X,+Y,-Y,+Z,-Z (D3D order),
texel centres mapped with the same face convention the sampler uses.  Mip m+1 is the
2x2 box average of mip m (a stand-in for Unity's specular convolution).  Deterministic: float64 math,
rounded to float32 once.
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache

import numpy as np


@dataclass(frozen=True, eq=False)
class Cubemap:
    face_size: int
    n_mips: int
    texels: np.ndarray  # flat float32

    def mip(self, m: int) -> np.ndarray:
        off = 0
        for k in range(m):
            s = max(1, self.face_size >> k)
            off += 6 * s * s * 4
        s = max(1, self.face_size >> m)
        return self.texels[off:off + 6 * s * s * 4].reshape(6, s, s, 4)


def _face_dirs(face: int, size: int) -> np.ndarray:
    c = (np.arange(size) + 0.5) / size * 2.0 - 1.0
    sc, tc = np.meshgrid(c, c)  # [y][x]: sc along x, tc along y
    one = np.ones_like(sc)
    # inverse of the sampler's (face, sc, tc) selection
    d = {
        0: (one, -tc, -sc), 1: (-one, -tc, sc), 2: (sc, one, tc),
        3: (sc, -one, -tc), 4: (sc, -tc, one), 5: (-sc, -tc, -one),
    }[face]
    v = np.stack(d, axis=-1)
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def _sky_radiance(d: np.ndarray) -> np.ndarray:
    y = d[..., 1]
    horizon = np.array([0.9, 0.85, 0.8])
    zenith = np.array([0.25, 0.45, 0.9])
    ground = np.array([0.18, 0.16, 0.14])
    t = np.clip(y, 0.0, 1.0)[..., None] ** 0.5
    sky = horizon * (1 - t) + zenith * t
    g = np.clip(-y * 4.0, 0.0, 1.0)[..., None]
    col = sky * (1 - g) + ground * g
    sun = np.array([0.35, 0.7, -0.62])
    sun /= np.linalg.norm(sun)
    cosang = np.clip(d @ sun, -1.0, 1.0)
    lobe = np.exp((cosang - 1.0) * 400.0)[..., None] * np.array([60.0, 55.0, 45.0])
    return col + lobe


@lru_cache(maxsize=4)
def synthetic_sky(face_size: int = 256) -> Cubemap:
    n_mips = int(np.log2(face_size)) + 1
    base = np.zeros((6, face_size, face_size, 4), dtype=np.float64)
    for f in range(6):
        base[f, :, :, :3] = _sky_radiance(_face_dirs(f, face_size))
        base[f, :, :, 3] = 1.0
    mips = [base]
    for _ in range(1, n_mips):
        p = mips[-1]
        s = p.shape[1] // 2
        mips.append(p.reshape(6, s, 2, s, 2, 4).mean(axis=(2, 4)))
    flat = np.concatenate([m.astype(np.float32).reshape(-1) for m in mips])
    return Cubemap(face_size, n_mips, flat)
