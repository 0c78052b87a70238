#!/usr/bin/env python3
"""Extract the benchmark scene constants from the reference's Unity files into a JSON fixture.

Reads (text only, no Unity):
  Assets/Scenes/Testing Scene.unity          the "Cornell Box" subtree: every child's name, active flag, local
                                             position / rotation / scale, built-in mesh (Plane / Cube) and its
                                             RayTracingMesh material block; the Dragon_87k instance's material
  Assets/URP-HighFidelity-Renderer.asset      the HalogenRenderFeature settings block (HalogenSettings)
and writes tests/golden/unity_scene.json.  Numbers are kept as the decimal strings the files hold, so a test can
compare them with the float32 constants of halogen/scenes.py exactly.  Unity scene files are YAML documents
introduced by `--- !u!<classID> &<fileID>`; each document body is plain YAML (yaml.safe_load).

Usage: python tools/extract_unity_scene.py [--reference /root/reference] [--out tests/golden/unity_scene.json]
"""
from __future__ import annotations

import argparse
import json
import re
from pathlib import Path

import yaml

ROOT = Path(__file__).resolve().parents[1]
SCENE = "Assets/Scenes/Testing Scene.unity"
RENDERER = "Assets/URP-HighFidelity-Renderer.asset"
BUILTIN_MESH = {10209: "Plane", 10202: "Cube", 10207: "Sphere"}  # Unity built-in mesh fileIDs (Library/unity default)
CLS_GAMEOBJECT, CLS_TRANSFORM = 1, 4


class _StrLoader(yaml.SafeLoader):
    """safe_load with every scalar kept as its source text (floats stay exact decimal strings)."""


_StrLoader.add_constructor("tag:yaml.org,2002:float", lambda l, n: l.construct_scalar(n))
_StrLoader.add_constructor("tag:yaml.org,2002:int", lambda l, n: l.construct_scalar(n))


def unity_documents(path: Path) -> dict[str, tuple[int, dict]]:
    """fileID -> (classID, document) of a Unity YAML file."""
    parts = re.split(r"^--- !u!(\d+) &(-?\d+).*$", path.read_text(), flags=re.M)
    docs = {}
    for i in range(1, len(parts), 3):
        docs[parts[i + 1]] = (int(parts[i]), yaml.load(parts[i + 2], Loader=_StrLoader) or {})
    return docs


def vec(d: dict, keys: str) -> list[str]:
    return [str(d[k]) for k in keys]


def material(mono: dict) -> dict:
    m = mono["material"]
    out = {}
    for k, v in m.items():
        out[k] = vec(v, "rgba") if isinstance(v, dict) else str(v)
    return out


def cornell_box(docs) -> dict:
    go = {fid: d["GameObject"] for fid, (c, d) in docs.items() if c == CLS_GAMEOBJECT and "GameObject" in d}
    tr = {fid: d["Transform"] for fid, (c, d) in docs.items() if c == CLS_TRANSFORM and "Transform" in d}
    owner = {str(c["component"]["fileID"]): fid for fid, g in go.items() for c in g.get("m_Component", [])}

    def node(tid: str) -> dict:
        t, g = tr[tid], go[owner[tid]]
        comps = [docs[str(c["component"]["fileID"])][1] for c in g["m_Component"]]
        out = {"name": g["m_Name"], "active": str(g["m_IsActive"]) == "1",
               "position": vec(t["m_LocalPosition"], "xyz"), "rotation": vec(t["m_LocalRotation"], "xyzw"),
               "scale": vec(t["m_LocalScale"], "xyz")}
        for comp in comps:
            if "MeshFilter" in comp:
                out["mesh"] = BUILTIN_MESH.get(int(comp["MeshFilter"]["m_Mesh"]["fileID"]), "other")
            if "MonoBehaviour" in comp and "material" in comp["MonoBehaviour"]:
                out["material"] = material(comp["MonoBehaviour"])
        out["children"] = [node(str(ch["fileID"])) for ch in t.get("m_Children", [])]
        return out

    roots = [tid for tid in tr if tid in owner and go[owner[tid]]["m_Name"] == "Cornell Box"]
    assert len(roots) == 1, roots
    return node(roots[0])


def dragon_material(docs) -> dict:
    """The RayTracingMesh on the Dragon_87k prefab instance (a stripped GameObject of a PrefabInstance whose
    modifications set m_Name: Dragon_87k)."""
    inst = [fid for fid, (c, d) in docs.items() if c == 1001 and any(
        m.get("propertyPath") == "m_Name" and m.get("value") == "Dragon_87k"
        for m in d["PrefabInstance"]["m_Modification"]["m_Modifications"])]
    assert len(inst) == 1, inst
    stripped = [fid for fid, (c, d) in docs.items() if c == CLS_GAMEOBJECT and "GameObject" in d
                and str(d["GameObject"].get("m_PrefabInstance", {}).get("fileID")) == inst[0]]
    monos = [d["MonoBehaviour"] for fid, (c, d) in docs.items() if "MonoBehaviour" in d
             and str(d["MonoBehaviour"].get("m_GameObject", {}).get("fileID")) in stripped
             and "material" in d["MonoBehaviour"]]
    assert len(monos) == 1, len(monos)
    return material(monos[0])


def renderer_settings(path: Path) -> dict:
    docs = unity_documents(path)
    feats = [d["MonoBehaviour"] for c, d in docs.values() if "MonoBehaviour" in d
             and d["MonoBehaviour"].get("m_Name") == "HalogenRenderFeature"]
    assert len(feats) == 1
    return {k: (str(v) if not isinstance(v, dict) else "<asset reference>") for k, v in feats[0]["settings"].items()}


def extract(reference: Path) -> dict:
    docs = unity_documents(reference / SCENE)
    return {"source": {"scene": SCENE, "renderer": RENDERER},
            "cornell_box": cornell_box(docs), "dragon_material": dragon_material(docs),
            "renderer_settings": renderer_settings(reference / RENDERER)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=str(ROOT / "tests" / "golden" / "unity_scene.json"))
    args = ap.parse_args()
    data = extract(Path(args.reference))
    Path(args.out).write_text(json.dumps(data, indent=1) + "\n")
    print(f"wrote {args.out}")


if __name__ == "__main__":
    main()
