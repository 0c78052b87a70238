"""The C# render pass over the C-ABI (bindings/csharp/HalogenRenderPass.cs) is a drop-in for the reference's
Assets/Scripts/Render Features/HalogenRenderPass.cs: the same class, base class and public members (signature by
signature, from tests/golden/renderpass_surface.json, which tools/extract_csharp_surface.py extracts from the
reference), every native call it makes declared in HalogenNative.cs and exported by the library's header, and the
scene records of HalogenStructs.cs field-for-field equal to the header's structs.  No C# toolchain exists in the
build image, so these textual checks stand in for compiling the binding."""
import json
import re
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import extract_csharp_surface as surf  # noqa: E402

CS_DIR = ROOT / "bindings" / "csharp"
PASS = (CS_DIR / "HalogenRenderPass.cs").read_text()
NATIVE = (CS_DIR / "HalogenNative.cs").read_text()
STRUCTS = (CS_DIR / "HalogenStructs.cs").read_text()
HEADER = (ROOT / "include" / "halogen_abi.h").read_text()
FIXTURE = ROOT / "tests" / "golden" / "renderpass_surface.json"


def test_public_surface_equals_the_reference():
    want = json.loads(FIXTURE.read_text())
    got = surf.surface(PASS)
    assert got["base"] == want["base"] == "ScriptableRenderPass"
    assert got["public_members"] == want["public_members"]


def test_native_calls_are_declared_and_exported():
    called = set(re.findall(r"HalogenNative\.(hg_\w+)\(", PASS))
    declared = set(re.findall(r"extern \w+ (hg_\w+)\(", NATIVE))
    exported = set(re.findall(r"^\w[\w\s\*]*?\b(hg_\w+)\(", HEADER, re.M))
    assert {"hg_create", "hg_upload_scene_gen", "hg_set_params", "hg_render", "hg_readback_begin_format",
            "hg_readback_end_data", "hg_set_accumulation", "hg_destroy",
            "hg_comm_init_all", "hg_comm_gather", "hg_comm_readback_begin", "hg_comm_readback_end"} <= called
    assert called <= declared <= exported, (called - declared, declared - exported)


C_TO_CS = {"hg_vec3": "Vector3", "hg_vec4": "Vector4", "hg_mat4": "Matrix4x4", "uint32_t": "uint", "int32_t": "int",
           "float": "float", "PackedRayMedium": "PackedRayMedium"}


def c_fields(name):
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), HEADER, re.S).group(1)
    out = []
    for decl in filter(None, (d.strip() for d in re.sub(r"/\*.*?\*/", "", body, flags=re.S).split(";"))):
        typ, names = decl.split(None, 1)
        out += [(C_TO_CS[typ], n.strip()) for n in names.split(",")]
    return out


def cs_fields(name):
    body = re.search(r"public struct %s\s*(?://[^\n]*)?\s*\{(.*?)\n\}" % name, STRUCTS, re.S).group(1)
    out = []
    for decl in filter(None, (d.strip() for d in re.sub(r"//[^\n]*", "", body).split(";"))):
        _, typ, names = decl.split(None, 2)
        out += [(typ, n.strip()) for n in names.split(",")]
    return out


@pytest.mark.parametrize("name", ["HalogenSphere", "HalogenMeshData", "PackedRayMedium", "PackedHalogenMaterial",
                                  "HalogenTriangle", "BVHEntry"])
def test_record_structs_match_header(name):
    assert cs_fields(name) == c_fields(name)
    assert re.search(r"\[StructLayout\(LayoutKind\.Sequential\)\]\s*public struct %s\b" % name, STRUCTS), name


@pytest.mark.skipif(not Path("/root/reference/Assets").exists(), reason="reference checkout absent (GPU box)")
def test_fixture_equals_fresh_extraction(tmp_path):
    out = tmp_path / "s.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "extract_csharp_surface.py"), "--out", str(out)], check=True,
                   capture_output=True)
    assert json.loads(out.read_text()) == json.loads(FIXTURE.read_text())
