"""BLAS build: the product builder (hg_build_blas, C++) equals the oracle's restatement of
BVHGenerator.GenerateMeshBVH (BVHGenerator.cs:13-134) node for node and in the reordered triangle list,
and the resulting trees satisfy the reference's structural rules."""
import ctypes as C

import numpy as np
import pytest

import hg_oracle
from halogen import abi
from halogen.scenes import dragon_mesh
from halogen.unity import mesh_bounds_min_max, unity_cube, unity_plane


def _build(fn, verts, tris, depth=32):
    verts = np.ascontiguousarray(verts, np.float32)
    idx = np.ascontiguousarray(tris, np.int32).copy()
    mn, mx = mesh_bounds_min_max(verts)
    mn, mx = np.ascontiguousarray(mn), np.ascontiguousarray(mx)
    cap = 2 * len(idx) + 2
    nodes = (abi.BVHEntry * cap)()
    fp = C.POINTER(C.c_float)
    n = fn(verts.ctypes.data, len(verts), idx.ctypes.data, len(idx), mn.ctypes.data_as(fp), mx.ctypes.data_as(fp),
           depth, C.cast(nodes, C.c_void_p), cap)
    assert n > 0
    return np.frombuffer(bytes(nodes)[: n * 32], dtype=np.uint8).reshape(n, 32), idx


def _check_tree(raw, n_tris, depth_cap=32):
    nodes = raw.view(np.uint32).reshape(-1, 8)
    idx_a, cnt = nodes[:, 0], nodes[:, 1]
    seen = np.zeros(n_tris, np.int32)
    stack = [(0, 0)]
    max_depth = 0
    while stack:
        g, d = stack.pop()
        max_depth = max(max_depth, d)
        if cnt[g] > 0:
            seen[idx_a[g]: idx_a[g] + cnt[g]] += 1
        else:
            assert idx_a[g] + 1 < len(nodes)
            stack += [(idx_a[g], d + 1), (idx_a[g] + 1, d + 1)]
    assert np.all(seen == 1), "every triangle in exactly one leaf"
    assert max_depth <= depth_cap
    return max_depth


@pytest.mark.parametrize("mesh", ["plane", "cube", "dragon8k", "dragon_x3"])
def test_product_builder_equals_oracle(built, mesh):
    if mesh == "plane":
        v, _, t = unity_plane()
    elif mesh == "cube":
        v, _, t = unity_cube()
    elif mesh == "dragon8k":
        v, _, t = dragon_mesh(1)
    else:
        v, _, t = dragon_mesh(3)
    a, ia = _build(abi.lib().hg_build_blas, v, t)
    b, ib = _build(hg_oracle.lib().hgo_build_blas, v, t)
    assert np.array_equal(a, b), "node arrays differ"
    assert np.array_equal(ia, ib), "triangle reorder differs"
    assert sorted(map(tuple, np.sort(ia, axis=1))) == sorted(map(tuple, np.sort(t, axis=1)))
    _check_tree(a, len(t))


def test_depth_cap_respected(built):
    v, _, t = dragon_mesh(1)
    a, _ = _build(abi.lib().hg_build_blas, v, t, depth=6)
    assert _check_tree(a, len(t), depth_cap=6) <= 6


def test_thin_box_pad_uses_unity_bounds(built):
    """A plane is flat in y: every child box gets the 1e-5 pad through Bounds' centre/extents round trip."""
    v, _, t = unity_plane()
    a, _ = _build(abi.lib().hg_build_blas, v, t)
    f = a.view(np.float32).reshape(-1, 8)
    assert f[0, 3] == f[0, 6] == 0.0  # root = mesh.bounds, no pad (BVHGenerator.cs:26-27)
    assert np.all(f[1:, 6] > f[1:, 3])  # children padded
