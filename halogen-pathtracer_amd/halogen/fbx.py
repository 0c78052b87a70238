"""Minimal binary-FBX (7.x) mesh reader: enough to read a triangle/polygon mesh with per-polygon-vertex
normals, which is what the reference's models are (Assets/Models/Dragon_8k.fbx: FBX 7400, normals
ByPolygonVertex).  Stands in for Unity's FBX importer, which the reference relies on
(RayTracingMesh.CacheRaytracingData reads GetTriangles/GetVertices/GetNormals of the imported mesh,
RayTracingMesh.cs:51-62).

Import convention (ours, documented in DESIGN.md §scene): polygons are fan-triangulated; every distinct
(position, normal) pair becomes one vertex (Unity splits vertices on normal seams the same way); the
FBX right-handed frame is mirrored to Unity's left-handed one by negating x (positions and normals) and
swapping two indices per triangle so cross(v1-v0, v2-v0) stays the outward normal.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np


def _read_props(buf: bytes, off: int, n: int):
    props = []
    for _ in range(n):
        t = chr(buf[off])
        off += 1
        if t in "YCIFDL":
            fmt = {"Y": "<h", "C": "<?", "I": "<i", "F": "<f", "D": "<d", "L": "<q"}[t]
            sz = struct.calcsize(fmt)
            props.append(struct.unpack_from(fmt, buf, off)[0])
            off += sz
        elif t in "fdlib":
            length, enc, clen = struct.unpack_from("<III", buf, off)
            off += 12
            raw = buf[off:off + clen]
            off += clen
            if enc == 1:
                raw = zlib.decompress(raw)
            dt = {"f": "<f4", "d": "<f8", "l": "<i8", "i": "<i4", "b": "<u1"}[t]
            props.append(np.frombuffer(raw, dtype=dt, count=length).copy())
        elif t in "SR":
            (length,) = struct.unpack_from("<I", buf, off)
            off += 4
            props.append(bytes(buf[off:off + length]))
            off += length
        else:
            raise ValueError(f"unknown FBX property type {t!r}")
    return props


def _read_nodes(buf: bytes, off: int, end: int, wide: bool):
    nodes = []
    hdr = "<QQQ" if wide else "<III"
    hsz = struct.calcsize(hdr)
    while off < end:
        end_off, n_props, _plen = struct.unpack_from(hdr, buf, off)
        if end_off == 0:  # NULL record terminates a nested list
            off += hsz + 1
            break
        name_len = buf[off + hsz]
        name = buf[off + hsz + 1: off + hsz + 1 + name_len].decode("ascii", "replace")
        p = off + hsz + 1 + name_len
        props = _read_props(buf, p, n_props)
        # skip props to find children: recompute offset by walking
        q = p
        for _ in range(n_props):
            t = chr(buf[q])
            q += 1
            if t in "YCIFDL":
                q += {"Y": 2, "C": 1, "I": 4, "F": 4, "D": 8, "L": 8}[t]
            elif t in "fdlib":
                q += 12 + struct.unpack_from("<III", buf, q)[2]
            else:
                q += 4 + struct.unpack_from("<I", buf, q)[0]
        children = _read_nodes(buf, q, end_off, wide) if q < end_off else []
        nodes.append((name, props, children))
        off = end_off
    return nodes


def _find(nodes, name):
    for n in nodes:
        if n[0] == name:
            yield n


def read_fbx_mesh(path: str):
    """Return (vertices (N,3) f32, normals (N,3) f32, triangles (M,3) i32) of the first Geometry node."""
    buf = open(path, "rb").read()
    if not buf.startswith(b"Kaydara FBX Binary"):
        raise ValueError("not a binary FBX")
    (version,) = struct.unpack_from("<I", buf, 23)
    nodes = _read_nodes(buf, 27, len(buf), wide=version >= 7500)
    objects = next(_find(nodes, "Objects"))
    geom = next(_find(objects[2], "Geometry"))
    g = {n[0]: n for n in geom[2]}
    pos = np.asarray(g["Vertices"][1][0], dtype=np.float64).reshape(-1, 3)
    pvi = np.asarray(g["PolygonVertexIndex"][1][0], dtype=np.int64)
    ln = {n[0]: n for n in g["LayerElementNormal"][2]}
    normals = np.asarray(ln["Normals"][1][0], dtype=np.float64).reshape(-1, 3)
    mapping = ln["MappingInformationType"][1][0].decode()
    ref = ln["ReferenceInformationType"][1][0].decode()
    if mapping != "ByPolygonVertex":
        raise ValueError(f"unsupported normal mapping {mapping}")
    if ref == "IndexToDirect":
        normals = normals[np.asarray(ln["NormalsIndex"][1][0], dtype=np.int64)]
    # polygons: a negative index closes a polygon (its value is ~index)
    corners_pos, corners_nrm = [], []
    poly = []
    for k, v in enumerate(pvi):
        poly.append(k)
        if v < 0:
            for i in range(1, len(poly) - 1):
                for c in (poly[0], poly[i], poly[i + 1]):
                    vi = pvi[c] if pvi[c] >= 0 else ~pvi[c]
                    corners_pos.append(pos[vi])
                    corners_nrm.append(normals[c])
            poly = []
    P = np.asarray(corners_pos, dtype=np.float64)
    Nn = np.asarray(corners_nrm, dtype=np.float64)
    # mirror to Unity's left-handed frame
    P[:, 0] *= -1.0
    Nn[:, 0] *= -1.0
    P32 = P.astype(np.float32)
    N32 = Nn.astype(np.float32)
    key = np.concatenate([P32.view(np.uint32), N32.view(np.uint32)], axis=1)
    uniq, inverse = np.unique(key, axis=0, return_inverse=True)
    verts = uniq[:, :3].copy().view(np.float32)
    norms = uniq[:, 3:].copy().view(np.float32)
    tris = inverse.reshape(-1, 3).astype(np.int32)
    tris = tris[:, [0, 2, 1]].copy()  # keep cross(v1-v0, v2-v0) outward after the mirror
    return verts, norms, tris
