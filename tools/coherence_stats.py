#!/usr/bin/env python3
"""Ray coherence of the descent loop (analysis build HG_COHERENCE_STATS=1, libraries under variants/): per node round
of the streaming traversal, how many distinct node records the loading lanes of the wave need (1-4 / 5-16 / 17-32 / >32).
  HALOGEN_LIB=variants/lib_coh.so python tools/coherence_stats.py [C3 C3F C2 ...]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "halogen-pathtracer_amd")]
from halogen import abi, render_pass as rp, scenes  # noqa: E402

for name in sys.argv[1:] or ["C3", "C3F"]:
    cfg = scenes.CONFIGS[name]
    settings = scenes.settings_for(cfg)
    s = rp.clamp_settings(settings)
    packed = cfg.build_scene().pack()
    cube = settings.environmentCubemap if s["UseEnvironmentCubemap"] else None
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), cube is not None)
    with abi.Context(0) as ctx:
        ctx.upload_scene(packed)
        if cube is not None:
            ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
        ctx.resize(cfg.width, cfg.height)
        ctx.set_params(params)
        ctx.set_option(abi.HG_OPT_COUNTERS, 1)
        ctx.render(8, True)
        ctx.synchronize()
        c = ctx.counters()
    h = c["shade_detail"]
    tot = max(sum(h), 1)
    print(json.dumps({"config": name, "node_rounds": c["node_rounds"], "hist_rounds": sum(h),
                      "distinct_records_share": {"1-4": h[0] / tot, "5-16": h[1] / tot, "17-32": h[2] / tot, ">32": h[3] / tot},
                      "descent_lane_util": c["aabb_tests"] / 2 / 64 / max(c["node_rounds"], 1)}))
