"""The benchmark scenes are built from the reference's own scene constants.

tests/golden/unity_scene.json is data extracted from the reference's Unity files by tools/extract_unity_scene.py
(Assets/Scenes/Testing Scene.unity: the "Cornell Box" subtree and the Dragon_87k material;
Assets/URP-HighFidelity-Renderer.asset: the HalogenRenderFeature settings).  The constants of halogen/scenes.py and
the HalogenSettings defaults must equal it exactly (float32 of the file's decimal text, -0 included).  When the
reference checkout is present, the fixture itself is re-extracted and compared."""
import dataclasses
import json
import struct
import subprocess
import sys
from pathlib import Path

import pytest

from halogen import render_pass as rp, scenes

ROOT = Path(__file__).resolve().parents[1]
FIXTURE = ROOT / "tests" / "golden" / "unity_scene.json"
REFERENCE = Path("/root/reference")


def f32_bits(x) -> int:
    return struct.unpack("<I", struct.pack("<f", float(x)))[0]


def same(py_values, file_values, what):
    assert len(py_values) == len(file_values), what
    for a, b in zip(py_values, file_values):
        assert f32_bits(a) == f32_bits(b), f"{what}: {a!r} != file {b!r}"


def same_material(mat, fm, what):
    same(mat.color, fm["color"], what + ".color")
    same(mat.specularColor, fm["specularColor"], what + ".specularColor")
    same(mat.subsurfaceColor, fm["subsurfaceColor"], what + ".subsurfaceColor")
    same(mat.emissionColor, fm["emissionColor"], what + ".emissionColor")
    for k in ("roughness", "metallic", "indexOfRefraction", "absorption", "emissionIntensity"):
        same([getattr(mat, k)], [fm[k]], f"{what}.{k}")
    assert mat.dielectricPriority == int(fm["dielectricPriority"]), what


@pytest.fixture(scope="module")
def fixture():
    return json.loads(FIXTURE.read_text())


def test_cornell_root(fixture):
    box = fixture["cornell_box"]
    assert box["name"] == "Cornell Box" and box["active"]
    same(scenes.CORNELL_ROOT, box["position"], "root position")
    same((0, 0, 0, 1), box["rotation"], "root rotation")
    same((1, 1, 1), box["scale"], "root scale")


def test_cornell_children_equal_the_scene_file(fixture):
    box = fixture["cornell_box"]
    by_name = {c["name"]: c for c in box["children"]}
    interior = by_name.pop("Basic Interior")
    same((0, 0, 0), interior["position"], "Basic Interior position")
    same((0, 0, 0, 1), interior["rotation"], "Basic Interior rotation")
    front = by_name.pop("Front Panel")
    assert front["active"] == scenes.CORNELL_FRONT_PANEL_ACTIVE
    ours = scenes.CORNELL_WALLS + [scenes.CORNELL_LIGHT]
    # the walls and the light, in the root's child order
    assert [o[0] for o in ours] == [c["name"] for c in box["children"] if c["name"] in by_name]
    for (name, mesh, pos, q, scale, mat), fc in zip(ours, (by_name[o[0]] for o in ours)):
        assert fc["active"] and fc["mesh"] == mesh, name
        same(pos, fc["position"], name + " position")
        same(q, fc["rotation"], name + " rotation")
        same(scale, fc["scale"], name + " scale")
        same_material(mat, fc["material"], name)
    assert [o[0] for o in scenes.CORNELL_INTERIOR] == [c["name"] for c in interior["children"]]
    for (name, mesh, pos, q, scale, mat), fc in zip(scenes.CORNELL_INTERIOR, interior["children"]):
        assert fc["active"] and fc["mesh"] == mesh, name
        same(pos, fc["position"], name + " position")
        same(q, fc["rotation"], name + " rotation")
        same(scale, fc["scale"], name + " scale")
        same_material(mat, fc["material"], name)


def test_dragon_material(fixture):
    same_material(scenes.DRAGON, fixture["dragon_material"], "Dragon_87k")


def test_renderer_settings_defaults(fixture):
    fs = fixture["renderer_settings"]
    d = rp.HalogenSettings()
    for f in dataclasses.fields(d):
        if f.name in ("environmentCubemap", "DebugMode"):
            continue
        v = getattr(d, f.name)
        want = fs[f.name]
        if isinstance(v, bool):
            assert v == (want == "1"), f.name
        elif isinstance(v, int):
            assert v == int(want), f.name
        else:
            same([v], [want], f.name)
    assert d.DebugMode == "None" and fs["DebugMode"] == "0"


def test_built_scene_uses_the_constants():
    """The packed C1 scene's meshes carry exactly the tabled transforms (world = root * local) and materials."""
    packed = scenes.cornell_box().pack()
    names = [o[0] for o in scenes.CORNELL_WALLS + [scenes.CORNELL_LIGHT] + scenes.CORNELL_INTERIOR]
    assert len(packed.meshes) == len(names)


@pytest.mark.skipif(not (REFERENCE / "Assets").exists(), reason="reference checkout absent (GPU box)")
def test_fixture_equals_fresh_extraction(tmp_path):
    out = tmp_path / "unity_scene.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "extract_unity_scene.py"), "--out", str(out)], check=True)
    assert json.loads(out.read_text()) == json.loads(FIXTURE.read_text())
