"""The distributed leaf test of the streaming kernel (hg_device.h leaf_dist) restated in numpy and
checked against the reference's sequential leaf loop (HalgoenCompute.compute:404-420, the order the oracle
follows).

A wave's lanes at a leaf own runs of (ray, triangle) pairs, numbered lane by lane by a prefix sum of the leaf
sizes; each 64-pair round, every pair's lane finds its owner (the lane whose run covers the pair), tests the
triangle against the owner's best_t of that round, and folds hits into the owner's key (t bits << 32 | triangle)
by a minimum; after the round an owner whose key came from that round takes the winner's u, v and facing.  The
claim: every owner ends with exactly the hit the sequential loop finds, ties included.  The per-triangle test is
the kernel's tri_accept in float32 with the same operation order (no fused multiply-add); the selection logic is
what is under test, so ties are forced with duplicated and edge-sharing triangles.
"""
import numpy as np

F = np.float32


def _cross(a, b):
    return np.array([F(a[1] * b[2]) - F(a[2] * b[1]), F(a[2] * b[0]) - F(a[0] * b[2]),
                     F(a[0] * b[1]) - F(a[1] * b[0])], dtype=F)


def _dot(a, b):
    return F(F(F(a[0] * b[0]) + F(a[1] * b[1])) + F(a[2] * b[2]))


def tri_test(lo, ld, v0, e1, e2):
    """triangle_intersection_doublesided (:307-355) as tri_accept computes it; the `t < best` part is left out."""
    pvec = _cross(ld, e2)
    det = _dot(pvec, e1)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        inv_det = F(F(1.0) / det)
        tvec = (lo - v0).astype(F)
        u = F(_dot(tvec, pvec) * inv_det)
        qvec = _cross(tvec, e1)
        v = F(_dot(ld, qvec) * inv_det)
        t = F(_dot(e2, qvec) * inv_det)
    ok = (not abs(det) < F(1e-8)) and not (u < 0 or u > 1) and not (v < 0 or F(u + v) > 1) and t > 0 and t > F(1e-4)
    return ok, t, u, v, det > 0


def sequential(lo, ld, tris, first, n, best_t):
    """The reference's loop: strict `<`, so the first triangle of minimal t wins."""
    best = (best_t, None, None, None, None)
    for k in range(n):
        ok, t, u, v, front = tris[first + k]
        if ok and t < best[0]:
            best = (t, u, v, first + k, front)
    return best


def distributed(owners, tris):
    """leaf_dist for one wave: owners[lane] = (best_t, first, n); returns each lane's final (t, u, v, tri, front)."""
    ns = np.array([o[2] for o in owners], dtype=np.int64)
    incl = np.cumsum(ns)
    total = int(incl[-1])
    start = incl - ns
    best = [(o[0], None, None, None, None) for o in owners]
    key = [None] * len(owners)
    for base in range(0, total, 64):
        # owner table: each run intersecting the round writes its lane id + 1 where it starts (or at 0); a running
        # max over the lanes then names every pair's owner
        tab = np.zeros(64, dtype=np.int64)
        for lane, (b, first, n) in enumerate(owners):
            if n and start[lane] < base + 64 and incl[lane] > base:
                tab[max(start[lane] - base, 0)] = lane + 1
        owner_of = np.maximum.accumulate(tab) - 1
        round_res = {}
        for j in range(64):
            p = base + j
            if p >= total:
                break
            o = int(owner_of[j])
            b, first, n = owners[o]
            assert start[o] <= p < incl[o]
            ti = first + (p - start[o])
            ok, t, u, v, front = tris[ti]
            if ok and t < best[o][0]:  # the owner's best_t of this round
                k = (int(np.asarray(t, dtype=F).view(np.uint32)) << 32) | ti
                if key[o] is None or k < key[o]:
                    key[o] = k
                round_res[(o, ti)] = (t, u, v, front)
        for o in range(len(owners)):  # owners whose key came from this round take the winner's u, v, facing
            if key[o] is not None and (o, key[o] & 0xFFFFFFFF) in round_res:
                t, u, v, front = round_res[(o, key[o] & 0xFFFFFFFF)]
                best[o] = (t, u, v, key[o] & 0xFFFFFFFF, front)
    return best


def _scene(rng, n_tris):
    """Triangles around the origin; a third are exact duplicates or share an edge with an earlier one."""
    verts = []
    for i in range(n_tris):
        r = rng.random()
        if i and r < 0.2:
            verts.append(verts[rng.integers(0, i)])  # duplicate: same t, u, v
        elif i and r < 0.35:
            a, b, _ = verts[rng.integers(0, i)]
            verts.append((b, a, rng.normal(0, 1, 3).astype(F)))  # shared edge, flipped
        else:
            verts.append(tuple(rng.normal(0, 1, 3).astype(F) for _ in range(3)))
    return verts


def _trial(rng, n_lanes, max_leaf):
    n_tris = 400
    verts = _scene(rng, n_tris)
    origin = (rng.normal(0, 0.2, 3) + np.array([0, 0, -6])).astype(F)
    target = rng.normal(0, 0.3, 3).astype(F)
    lo = origin
    ld = (target - origin).astype(F)  # unnormalised, as the kernel's local-space direction
    owners, rays = [], []
    for lane in range(n_lanes):
        if rng.random() < 0.3:
            owners.append((F(np.inf), 0, 0))  # not at a leaf
            continue
        n = int(rng.integers(1, max_leaf + 1))
        first = int(rng.integers(0, n_tris - n))
        best_t = F(np.inf) if rng.random() < 0.7 else F(rng.uniform(3, 9))
        owners.append((best_t, first, n))
    # one ray per wave keeps the numpy cost low; every lane still has its own leaf and best_t
    tris = [tri_test(lo, ld, v0, (v1 - v0).astype(F), (v2 - v0).astype(F)) for v0, v1, v2 in verts]
    got = distributed(owners, tris)
    for lane, (best_t, first, n) in enumerate(owners):
        want = sequential(lo, ld, tris, first, n, best_t)
        g = got[lane]
        assert (g[3], g[4]) == (want[3], want[4]), (lane, g, want)
        assert np.asarray(g[0], F).view(np.uint32) == np.asarray(want[0], F).view(np.uint32)
        if want[3] is not None:
            assert (np.asarray(g[1], F).view(np.uint32), np.asarray(g[2], F).view(np.uint32)) == \
                   (np.asarray(want[1], F).view(np.uint32), np.asarray(want[2], F).view(np.uint32))


def test_leaf_exchange_equals_sequential_loop_small_leaves():
    rng = np.random.default_rng(7)
    for _ in range(60):
        _trial(rng, 64, 5)  # the reference's leaves (<= 5 triangles): up to 320 pairs, several rounds


def test_leaf_exchange_equals_sequential_loop_large_leaves():
    rng = np.random.default_rng(11)
    for _ in range(10):
        _trial(rng, 64, 201)  # depth-capped leaves as in the dragon (up to 201 triangles)


def test_leaf_exchange_ties_resolve_to_first_triangle():
    """Two identical triangles in one leaf: the sequential loop keeps the first, and so must the key minimum."""
    v0, v1, v2 = (np.array(x, dtype=F) for x in ([-1, -1, 0], [1, -1, 0], [0, 1, 0]))
    lo, ld = np.array([0, 0, -5], dtype=F), np.array([0, 0, 1], dtype=F)
    tri = tri_test(lo, ld, v0, (v1 - v0).astype(F), (v2 - v0).astype(F))
    assert tri[0]
    tris = [tri, tri, tri]
    got = distributed([(F(np.inf), 0, 3)], tris)[0]
    assert got[3] == 0 == sequential(lo, ld, tris, 0, 3, F(np.inf))[3]
