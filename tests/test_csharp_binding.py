"""The C# P/Invoke binding (bindings/csharp/HalogenNative.cs) stays in step with include/halogen_abi.h: every
exported function is declared, the uniform / counter structs have the header's fields in the header's order with
the matching C# types, and the option / kernel constants carry the header's values.  (No C# toolchain exists in
the build image, so this textual check stands in for compiling it.)"""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HEADER = (ROOT / "include" / "halogen_abi.h").read_text()
CS = (ROOT / "bindings" / "csharp" / "HalogenNative.cs").read_text()

C_TO_CS = {"hg_mat4": "Matrix4x4", "hg_vec4": "Vector4", "int32_t": "int", "uint32_t": "uint",
           "uint64_t": "ulong", "double": "double", "float": "float"}


def c_struct(name):
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), HEADER, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        typ, names = decl.split(None, 1)
        for n in names.split(","):
            n = n.strip()
            if "[" in n:  # fixed-size array member: uint64_t x[4] <-> public ulong[] x (ByValArray)
                fields.append((typ + "[]", n[:n.index("[")]))
            else:
                fields.append((typ, n))
    return fields


def cs_struct(name):
    body = re.search(r"public struct %s\s*\{(.*?)\n    \}" % name, CS, re.S).group(1)
    body = re.sub(r"//[^\n]*", "", body)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        decl = re.sub(r"^\[MarshalAs\(UnmanagedType\.ByValArray, SizeConst = \d+\)\]\s*", "", decl)
        _, typ, names = decl.split(None, 2)
        fields += [(typ, n.strip()) for n in names.split(",")]
    return fields


def test_every_export_is_declared():
    exports = set(re.findall(r"^\w[\w\s\*]*?\b(hg_\w+)\(", HEADER, re.M))
    declared = set(re.findall(r"extern \w+ (hg_\w+)\(", CS))
    assert exports and exports == declared, (exports - declared, declared - exports)


def test_struct_layouts_match_header():
    for c_name, cs_name in (("hg_params", "HgParams"), ("hg_counters", "HgCounters")):
        c_fields, cs_fields = c_struct(c_name), cs_struct(cs_name)
        assert [n for _, n in c_fields] == [n for _, n in cs_fields], c_name
        cs_type = lambda t: C_TO_CS[t[:-2]] + "[]" if t.endswith("[]") else C_TO_CS[t]
        assert [cs_type(t) for t, _ in c_fields] == [t for t, _ in cs_fields], c_name


def test_constants_match_header():
    header_consts = dict((k, int(v)) for k, v in re.findall(r"\b(HG_(?:KERNEL|OPT|SELFTEST)_\w+) = (\d+)", HEADER))
    cs_consts = dict((k, int(v)) for k, v in re.findall(r"\b(HG_(?:KERNEL|OPT|SELFTEST)_\w+) = (\d+)", CS))
    assert header_consts and header_consts == cs_consts
