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


def _build_mt(threads):
    def fn(*args):
        return abi.lib().hg_build_blas_mt(*args, threads)
    return fn


def _shuffled(t, seed):
    return np.random.default_rng(seed).permutation(np.asarray(t)).astype(np.int32)


@pytest.mark.parametrize("threads", [2, 5, 16])
@pytest.mark.parametrize("mesh", ["dragon_x3", "dragon_x3_shuffled", "grid_ties"])
def test_parallel_builder_equals_sequential(built, mesh, threads):
    """hg_build_blas_mt (level-parallel, rank-parallel partition of large nodes) returns the node array and the
    reordered triangle list of the sequential hg_build_blas."""
    if mesh.startswith("dragon"):
        v, _, t = dragon_mesh(3)  # 78,408 triangles: the top levels take the rank-parallel partition
        if mesh.endswith("shuffled"):
            t = _shuffled(t, 3)
    else:  # a lattice of coincident centroids and +-0 coordinates: ties on the split plane and in the folds
        g = np.stack(np.meshgrid(np.arange(-20, 21), np.arange(-20, 21), np.arange(-20, 21)), -1).reshape(-1, 3)
        v = (g * 0.5).astype(np.float32)
        v[v == 0] = -0.0
        rng = np.random.default_rng(5)
        t = rng.integers(0, len(v), size=(60000, 3)).astype(np.int32)
        t[::7] = t[::7, :1]  # degenerate triangles: all three vertices equal
    a, ia = _build(abi.lib().hg_build_blas, v, t)
    b, ib = _build(_build_mt(threads), v, t)
    assert np.array_equal(a, b), "node arrays differ"
    assert np.array_equal(ia, ib), "triangle reorder differs"


def test_parallel_partition_rule_small_cases(built):
    """The rank rule of the parallel partition (hg_host.cpp) against the two-pointer loop it restates, on every
    left/right pattern of length <= 10 (the C++ path only takes it for large nodes)."""
    import itertools

    def two_pointer(a, left):
        a = list(a); i, j = 0, len(a) - 1
        while i <= j:
            if left[a[i]]:
                i += 1
            else:
                a[i], a[j] = a[j], a[i]; j -= 1
        return a

    def rank_rule(a, left):
        n = len(a); L = [left[v] for v in a]; A = sum(L)
        P = [x for x in range(A) if not L[x]]
        Q = [x for x in range(n - 1, A - 1, -1) if L[x]]
        q = lambda k: n if k == 0 else Q[k - 1]
        out = [None] * n
        for x in range(n):
            if x < A:
                out[x if L[x] else q(P.index(x)) - 1] = a[x]
            elif L[x]:
                out[P[Q.index(x)]] = a[x]
            else:
                out[q(len(P)) - 1 if x == A else x - 1] = a[x]
        return out

    for n in range(11):
        for pattern in itertools.product([False, True], repeat=n):
            a = list(range(n))
            assert rank_rule(a, pattern) == two_pointer(a, pattern)
