"""Convert the reference's Assets/Models/Dragon_8k.fbx into assets/dragon_8k.npz (run in the build container only;
/root/reference does not exist on the GPU box).  The .npz holds plain float32/int32 arrays (no pickles):
vertices (N,3), normals (N,3), triangles (M,3) after the import convention of halogen/fbx.py."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "halogen-pathtracer_amd"))
from halogen.fbx import read_fbx_mesh  # noqa: E402

src = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/Assets/Models/Dragon_8k.fbx")
v, n, t = read_fbx_mesh(str(src))
out = ROOT / "assets" / "dragon_8k.npz"
np.savez_compressed(out, vertices=v, normals=n, triangles=t)
print(f"{src.name}: {len(v)} vertices, {len(t)} triangles -> {out} ({out.stat().st_size} bytes)")
