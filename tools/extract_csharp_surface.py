#!/usr/bin/env python3
"""Extract the public surface of the reference's HalogenRenderPass class (Assets/Scripts/Render Features/
HalogenRenderPass.cs) into tests/golden/renderpass_surface.json: the base class and every public / public override
member's signature (return type, name, parameter types and modifiers), whitespace-normalised.  The same parser,
applied to bindings/csharp/HalogenRenderPass.cs, must give the same list (tests/test_csharp_render_pass.py).

Usage: python tools/extract_csharp_surface.py [--reference /root/reference] [--out tests/golden/renderpass_surface.json]
"""
from __future__ import annotations

import argparse
import json
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
REF_FILE = "Assets/Scripts/Render Features/HalogenRenderPass.cs"
CLASS = "HalogenRenderPass"


def strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def class_body(src: str, name: str) -> tuple[str, str]:
    """(base class, body text) of `class name : Base { ... }` (brace matched)."""
    m = re.search(r"\bclass\s+%s\s*:\s*([A-Za-z_][\w.]*)\s*\{" % name, src)
    if not m:
        raise ValueError(f"class {name} not found")
    depth, i = 1, m.end()
    while depth:
        depth += {"{": 1, "}": -1}.get(src[i], 0)
        i += 1
    return m.group(1), src[m.end():i - 1]


def top_level(body: str) -> str:
    """The class body with every nested brace block removed (member bodies, initialisers)."""
    out, depth = [], 0
    for ch in body:
        if ch == "{":
            depth += 1
            if depth == 1:
                out.append(";")
            continue
        if ch == "}":
            depth -= 1
            continue
        if depth == 0:
            out.append(ch)
    return "".join(out)


def param_sig(params: str) -> list[str]:
    sig = []
    for p in filter(None, (x.strip() for x in params.split(","))):
        words = p.split("=")[0].split()
        sig.append(" ".join(words[:-1]))  # modifiers + type, without the parameter name
    return sig


def surface(src: str, name: str = CLASS) -> dict:
    base, body = class_body(strip_comments(src), name)
    members = []
    for decl in top_level(body).split(";"):
        decl = " ".join(decl.split())
        m = re.match(r"public\s+(override\s+|virtual\s+|static\s+)?(?:([\w<>\[\],.]+)\s+)?(~?\w+)\s*\((.*)\)$", decl)
        if not m:
            continue
        mod, ret, mname, params = m.groups()
        members.append({"name": mname, "returns": ret or "", "modifier": (mod or "").strip(),
                        "params": param_sig(params)})
    members.sort(key=lambda d: (d["name"], d["params"]))
    return {"class": name, "base": base, "public_members": members}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=str(ROOT / "tests" / "golden" / "renderpass_surface.json"))
    a = ap.parse_args()
    data = surface((Path(a.reference) / REF_FILE).read_text())
    data["source"] = REF_FILE
    Path(a.out).write_text(json.dumps(data, indent=1) + "\n")
    print(json.dumps(data, indent=1))


if __name__ == "__main__":
    main()
