"""The C-ABI boundary: struct layouts byte-identical to the reference's C# structs (RP:10-76) and the
library exporting exactly the entry points include/halogen_abi.h declares.  CPU only (no compute calls)."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

from halogen import abi

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "halogen_abi.h"

# Marshal.SizeOf of the reference structs (RP:163-167)
REF_SIZES = {"HalogenSphere": 44, "HalogenMeshData": 164, "PackedHalogenMaterial": 84, "HalogenTriangle": 72,
             "BVHEntry": 32, "PackedRayMedium": 24}


def test_reference_struct_sizes(built):
    for name, size in REF_SIZES.items():
        assert C.sizeof(getattr(abi, name)) == size, name


def _c_layout():
    """sizeof/offsetof of every ABI struct field as compiled by gcc from the header."""
    structs = {"HalogenSphere": abi.HalogenSphere, "HalogenMeshData": abi.HalogenMeshData,
               "PackedRayMedium": abi.PackedRayMedium, "PackedHalogenMaterial": abi.PackedHalogenMaterial,
               "HalogenTriangle": abi.HalogenTriangle, "BVHEntry": abi.BVHEntry, "hg_params": abi.HgParams,
               "hg_counters": abi.HgCounters}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "halogen_abi.h"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = Path("/tmp/hg_layout_probe.c")
    src.write_text("\n".join(lines))
    exe = Path("/tmp/hg_layout_probe")
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    res = {}
    for ln in out.splitlines():
        s, f, v = ln.split()
        res[(s, f)] = int(v)
    return structs, res


def test_ctypes_mirror_matches_header(built):
    structs, res = _c_layout()
    for cname, py in structs.items():
        assert C.sizeof(py) == res[(cname, "size")], cname
        for f, _ in py._fields_:
            assert getattr(py, f).offset == res[(cname, f)], (cname, f)


def test_library_exports_every_declared_symbol(built):
    declared = sorted(set(re.findall(r"\b(hg_[a-z_]+)\s*\(", HEADER.read_text())))
    assert sorted(abi.EXPORTS) == declared
    so = abi.LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", str(so)], check=True, capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (hg_[a-z_]+)\b", out))
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    L = abi.lib()  # loads, binds every signature
    assert L.hg_abi_version() == 6


def test_error_codes_match_header(built):
    declared = {k: int(v) for k, v in re.findall(r"\b(HG_E_\w+) = (-\d+)", HEADER.read_text())}
    assert declared and all(getattr(abi, k) == v for k, v in declared.items()), declared


def test_no_gpu_is_a_loud_error(built):
    """Product path has no CPU fallback: without a device, hg_create fails and Context raises."""
    if abi.gpu_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(abi.HalogenError):
        abi.Context(0)
