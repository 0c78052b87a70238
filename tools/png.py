"""Tiny PNG writer (no PIL in the image) for looking at renders: sRGB-ish gamma, clamp, y flipped so row 0
(NDC y = -1, the bottom of the view) ends up at the bottom of the picture."""
import struct
import zlib

import numpy as np


def save_png(path, rgba: np.ndarray, exposure: float = 1.0):
    img = np.clip(rgba[..., :3] * exposure, 0.0, 1.0) ** (1.0 / 2.2)
    img = (img[::-1] * 255.0 + 0.5).astype(np.uint8)
    h, w, _ = img.shape
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))

    def chunk(t, d):
        c = struct.pack(">I", len(d)) + t + d
        return c + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
                + chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))
