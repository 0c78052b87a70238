"""Diagnose a variant library on golden cases: differing pixels, their 8x8-tile lane pattern, counter mismatches.

  HALOGEN_LIB=variants/lib_x.so python tools/diag_golden.py [kernel] [case ...]   (kernel: regen, stream, ...)
"""
import json, sys
from pathlib import Path
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "halogen-pathtracer_amd"); sys.path.insert(0, "oracle")
import cases
from test_gpu_parity import gpu_render
GOLD = Path("tests/golden")
kernel = sys.argv[1] if len(sys.argv) > 1 else "auto"
for name in (sys.argv[2:] or ["c1_32_aperture", "c1_64"]):
    meta = json.loads((GOLD / f"{name}.json").read_text())
    packed, params, cube, frames, acc = cases.setup(name)
    img, cnt = gpu_render(packed, params, frames, acc, cube, kernel=kernel)
    ref = np.load(GOLD / f"{name}.npz")["image"]
    d = (img.view(np.uint32) != ref.view(np.uint32)).any(axis=2)
    ys, xs = np.nonzero(d)
    print(name, "differing pixels", int(d.sum()), "of", d.size)
    if len(ys):
        print("  first", list(zip(ys[:10].tolist(), xs[:10].tolist())))
        print("  lanes", sorted(set(((ys % 8) * 8 + xs % 8).tolist()))[:64])
        print("  max abs diff", float(np.abs(img - ref).max()))
    print("  counters", {k: (cnt[k], v) for k, v in meta["counters"].items() if cnt[k] != v})
