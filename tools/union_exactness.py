#!/usr/bin/env python3
"""DESIGN §10 lever 5 (parent-relative child-pair records) needs every inner node's box to be exactly the union of its
children's boxes: then each of the six (axis, side) bounds is attained by one child, and a record could store only the
other six values.  BVHGenerator stores every box through Unity Bounds (centre / extents, BVHGenerator.cs:171-183), which
re-derives min / max with rounding, so the property can fail.  This counts it on the C3 dragon's BLAS (the product
builder, hg_build_blas_mt, node for node the reference's).
    python3 tools/union_exactness.py"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "halogen-pathtracer_amd"))
from halogen import scenes  # noqa: E402

s = scenes.dragon_cornell()
m = max(s.meshes, key=lambda o: o.triangle_count)
raw = np.frombuffer(bytes(m.bvh), dtype=np.dtype([("a", "<u4"), ("n", "<u4"), ("lo", "<f4", 3), ("hi", "<f4", 3)]))
inner = np.nonzero(raw["n"] == 0)[0]
a = raw["a"][inner].astype(np.int64)
b = a + 1  # children are appended A then B (BVHGenerator.cs:101-117)
box = lambda i: np.concatenate([raw["lo"][i], raw["hi"][i]], 1)  # noqa: E731
P, A, B = box(inner), box(a), box(b)
eq = (P == A) | (P == B)
inside = ((A[:, :3] >= P[:, :3]) & (A[:, 3:] <= P[:, 3:])).all(1) & ((B[:, :3] >= P[:, :3]) & (B[:, 3:] <= P[:, 3:])).all(1)
print(f"dragon BLAS: {len(raw)} nodes, {len(inner)} inner")
print(f"inner nodes whose 6 bounds are each attained exactly by a child: {eq.all(1).mean():.4f}")
print("per bound (min x, y, z, max x, y, z):", " ".join(f"{v:.4f}" for v in eq.mean(0)))
print(f"inner nodes with both children inside the parent box: {inside.mean():.4f}")
