"""Generate tests/golden/<case>.npz + .json with the CPU oracle (run in the build container).  A golden holds the
accumulated float32 image, the work counters, and sha256 digests of the packed scene and the image, so both a
changed scene builder and a changed result are detected.  Usage: python tools/make_goldens.py [case ...]"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in ("halogen-pathtracer_amd", "oracle", "tests"):
    sys.path.insert(0, str(ROOT / p))
import cases  # noqa: E402
import hg_oracle  # noqa: E402

out_dir = ROOT / "tests" / "golden"
names = sys.argv[1:] or list(cases.CASES)
for name in names:
    packed, params, cube, frames, acc_flag = cases.setup(name)
    img, cnt = hg_oracle.render(packed, params, frames, acc_flag, cubemap=cube)
    np.savez_compressed(out_dir / f"{name}.npz", image=img)
    meta = {"case": name, "frames": frames, "accumulate": acc_flag, "counters": {k: int(v) for k, v in cnt.items()
            if k not in ("kernel_ms", "launches")}, "scene_sha256": cases.packed_digest(packed),
            "image_sha256": hashlib.sha256(img.tobytes()).hexdigest(), "shape": list(img.shape)}
    (out_dir / f"{name}.json").write_text(json.dumps(meta, indent=1))
    print(name, img.shape, meta["counters"]["paths"], meta["image_sha256"][:16])
