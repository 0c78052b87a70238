"""How often does a BVH descent step keep 0, 1 or 2 children (the exact test, t < closest)?  The bound on any exact
pre-filter of child boxes: a conservative quantized box rejects at most the children the exact
test rejects, and only a step that rejects BOTH avoids fetching exact boxes.  Oracle (test infra) on row bands of a
BASELINE config, frame 1..F."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "halogen-pathtracer_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

import cases  # noqa: E402
import hg_oracle  # noqa: E402
from halogen import render_pass as rp, scenes  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C3"
cfg = scenes.CONFIGS[cfg_name]
settings = scenes.settings_for(cfg)
s = rp.clamp_settings(settings)
packed = cases._scene(cfg.scene, 10)
cube = settings.environmentCubemap if s["UseEnvironmentCubemap"] else None
params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), cube is not None)
W, H = cfg.width, cfg.height
hg_oracle.visit_stats(reset=True)
tot = {"paths": 0, "aabb_tests": 0}
for y in np.linspace(0, H - 2, 9).astype(int):
    _, cnt = hg_oracle.render(packed, params, 2, True, cubemap=cube, pix_range=(int(y) * W, (int(y) + 2) * W), threads=8, stats=True)
    tot["paths"] += cnt["paths"]
    tot["aabb_tests"] += cnt["aabb_tests"]
v = hg_oracle.visit_stats()
inner = np.array(v["inner"], float)
root = np.array(v["root"], float)
print(json.dumps({"config": cfg_name, "bands": "9 x 2 rows, 2 frames", **tot, "root_visits_by_kept_children": v["root"],
                  "inner_visits_by_kept_children": v["inner"],
                  "inner_frac": (inner / inner.sum()).round(4).tolist(),
                  "root_frac": (root / root.sum()).round(4).tolist()}))
