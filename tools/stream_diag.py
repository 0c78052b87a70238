"""Diagnose stream-kernel determinism on the deep dragon scene: split / tiling / descent threshold vs regen."""
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "halogen-pathtracer_amd"))
from halogen import abi, render_pass as rp, scenes

cfg = scenes.CONFIGS["C3"].resized(128, 96, 1)
packed = scenes.dragon_cornell(10).pack()
s = rp.clamp_settings(scenes.settings_for(cfg))
params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), False)
W, H = 128, 96

def render(kernel, frames=8, split=-1, tiling=None, dt=-2):
    img = np.full((H, W, 4), np.nan, np.float32)
    parts = [tiling] if tiling else [None]
    if tiling:
        parts = [(r, tiling) for r in range(tiling)]
    for part in parts:
        with abi.Context(0) as ctx:
            ctx.set_option(abi.HG_OPT_KERNEL, kernel)
            if split >= 0: ctx.set_option(abi.HG_OPT_FRAME_SPLIT, split)
            if dt >= -1: ctx.set_option(abi.HG_OPT_DESCENT_T, dt)
            ctx.upload_scene(packed); ctx.resize(W, H)
            if part: ctx.set_tiling(*part)
            ctx.set_params(params); ctx.render(frames, True)
            p = np.full((H, W, 4), np.nan, np.float32); ctx.readback(W, H, p)
            m = ~np.isnan(p); img[m] = p[m]
    return img

def same(a, b): return int((a.view(np.uint32) != b.view(np.uint32)).sum())
ref = render(abi.HG_KERNEL_MEGA_REGEN, split=1)
print("regen split auto vs 1:", same(render(abi.HG_KERNEL_MEGA_REGEN), ref))
S = abi.HG_KERNEL_MEGA_STREAM
print("stream split 1:", same(render(S, split=1), ref))
print("stream split 1 dt0:", same(render(S, split=1, dt=0), ref))
print("stream split auto:", same(render(S), ref))
print("stream split 3:", same(render(S, split=3), ref))
print("stream tiling 2 split 1:", same(render(S, split=1, tiling=2), ref))
print("stream split 1 repeat:", same(render(S, split=1), render(S, split=1)))
