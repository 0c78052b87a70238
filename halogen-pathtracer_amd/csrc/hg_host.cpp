// hg_host.cpp — host-side data producers of the Halogen hot path (product code).
//
// The reference builds its GPU buffers in C#:
//   BVHGenerator.GenerateMeshBVH        Assets/Scripts/BVHGenerator.cs:13-134   -> hg_build_blas
//   Bounds arithmetic (SetMinMax/min/max) BVHGenerator.cs:154-186, RayTracingMesh.cs:106-117 -> hg_unity_bounds
//   RayTracingMesh.UpdateTriangleList   Assets/Scripts/RayTracingMesh.cs:70-87   -> hg_pack_triangles
// The C# side stays C# where a runtime exists; these C++ equivalents serve every other
// caller.  They must produce the SAME node array as the C# code (triangle order and traversal counts
// depend on it), so the float arithmetic is kept in the reference's order: Unity's Bounds stores
// centre/extents, so every min/max goes through  e=(max-min)*0.5, c=min+e, min=c-e, max=c+e.
// Compiled with -ffp-contract=off.
#include <cstdint>
#include <cstring>
#include <limits>
#include <utility>
#include <vector>

#include "halogen_abi.h"

namespace {

constexpr float kAabbEpsilon = 0.00001f;  // RayTracingMesh.AABBEpsilon (RayTracingMesh.cs:11)
constexpr uint32_t kMaxNodeTriangleCount = 5;  // BVHGenerator.maxNodeTriangleCount (BVHGenerator.cs:8)

struct Vec3 {
    float v[3];
    float& operator[](int k) { return v[k]; }
    float operator[](int k) const { return v[k]; }
};

// UnityEngine.Bounds: centre + extents storage.
struct UnityBounds {
    Vec3 center, extents;
    static UnityBounds FromMinMax(const Vec3& mn, const Vec3& mx) {  // Bounds.SetMinMax
        UnityBounds b;
        for (int k = 0; k < 3; ++k) {
            b.extents[k] = (mx[k] - mn[k]) * 0.5f;
            b.center[k] = mn[k] + b.extents[k];
        }
        return b;
    }
    Vec3 Min() const { Vec3 r; for (int k = 0; k < 3; ++k) r[k] = center[k] - extents[k]; return r; }
    Vec3 Max() const { Vec3 r; for (int k = 0; k < 3; ++k) r[k] = center[k] + extents[k]; return r; }
    Vec3 Size() const { Vec3 r; for (int k = 0; k < 3; ++k) r[k] = extents[k] * 2.0f; return r; }
    // `bounds.max += Vector3.one * AABBEpsilon` when any side is thinner than the epsilon
    void PadIfThin() {
        Vec3 s = Size();
        if (s[0] < kAabbEpsilon || s[1] < kAabbEpsilon || s[2] < kAabbEpsilon) {
            Vec3 mx = Max();
            for (int k = 0; k < 3; ++k) mx[k] = mx[k] + kAabbEpsilon * 1.0f;
            *this = FromMinMax(Min(), mx);
        }
    }
};

BVHEntry MakeEntry(const Vec3& mn, const Vec3& mx, uint32_t indexA, uint32_t count) {
    BVHEntry e;
    e.indexA = indexA;
    e.triangleCount = count;
    e.boundingCornerA = {mn[0], mn[1], mn[2]};
    e.boundingCornerB = {mx[0], mx[1], mx[2]};
    return e;
}

// calculateBounds (BVHGenerator.cs:154-186); Vector3.Min/Max are Mathf.Min/Max (a<b?a:b / a>b?a:b).
UnityBounds TriangleRangeBounds(uint32_t start, uint32_t count, const int32_t* idx, const float* V) {
    const float inf = std::numeric_limits<float>::infinity();
    Vec3 mn{{inf, inf, inf}}, mx{{-inf, -inf, -inf}};
    for (uint64_t i = start; i < uint64_t(start) + count; ++i) {
        for (int c = 0; c < 3; ++c) {
            const float* p = V + 3 * int64_t(idx[3 * i + c]);
            for (int k = 0; k < 3; ++k) {
                mn[k] = mn[k] < p[k] ? mn[k] : p[k];
                mx[k] = mx[k] > p[k] ? mx[k] : p[k];
            }
        }
    }
    UnityBounds b = UnityBounds::FromMinMax(mn, mx);
    b.PadIfThin();
    return b;
}

}  // namespace

extern "C" void hg_unity_bounds(const float in_min[3], const float in_max[3], int32_t pad_if_thin, float out_min[3],
                                float out_max[3]) {
    UnityBounds b = UnityBounds::FromMinMax(Vec3{{in_min[0], in_min[1], in_min[2]}},
                                            Vec3{{in_max[0], in_max[1], in_max[2]}});
    if (pad_if_thin) b.PadIfThin();
    Vec3 mn = b.Min(), mx = b.Max();
    for (int k = 0; k < 3; ++k) {
        out_min[k] = mn[k];
        out_max[k] = mx[k];
    }
}

extern "C" int64_t hg_build_blas(const float* V, int32_t n_vertices, int32_t* idx, int32_t n_tris,
                                 const float root_min[3], const float root_max[3], int32_t max_hierarchy_depth,
                                 BVHEntry* out_nodes, int64_t max_nodes) {
    if (!V || !idx || n_tris < 0 || n_vertices < 0 || !root_min || !root_max) return HG_E_INVALID;
    for (int64_t i = 0; i < 3 * int64_t(n_tris); ++i)
        if (idx[i] < 0 || idx[i] >= n_vertices) return HG_E_INVALID;

    std::vector<BVHEntry> nodes;
    nodes.reserve(size_t(2) * size_t(n_tris) + 1);
    {
        // root = initializeLeafEntry(mesh.bounds.min, mesh.bounds.max, 0, n) — mesh.bounds has no pad
        UnityBounds rb = UnityBounds::FromMinMax(Vec3{{root_min[0], root_min[1], root_min[2]}},
                                                 Vec3{{root_max[0], root_max[1], root_max[2]}});
        nodes.push_back(MakeEntry(rb.Min(), rb.Max(), 0, uint32_t(n_tris)));
    }
    // triangle centroids (v0+v1+v2)/3, kept in the same permutation as the index triples
    std::vector<float> cen(size_t(n_tris) * 3);
    for (int64_t t = 0; t < n_tris; ++t) {
        const float* a = V + 3 * int64_t(idx[3 * t]);
        const float* b = V + 3 * int64_t(idx[3 * t + 1]);
        const float* c = V + 3 * int64_t(idx[3 * t + 2]);
        for (int k = 0; k < 3; ++k) cen[3 * t + k] = ((a[k] + b[k]) + c[k]) / 3.0f;
    }
    // breadth-first, one queue per depth (BVHGenerator.cs:40-129)
    std::vector<int32_t> queue{0}, next;
    for (int depth = 1; depth <= max_hierarchy_depth && !queue.empty(); ++depth) {
        for (int32_t entry : queue) {
            BVHEntry cur = nodes[size_t(entry)];
            const uint32_t first = cur.indexA, count = cur.triangleCount;
            const float size[3] = {cur.boundingCornerB.x - cur.boundingCornerA.x,
                                   cur.boundingCornerB.y - cur.boundingCornerA.y,
                                   cur.boundingCornerB.z - cur.boundingCornerA.z};
            const float lo[3] = {cur.boundingCornerA.x, cur.boundingCornerA.y, cur.boundingCornerA.z};
            const int axis = size[0] > size[1] ? (size[0] > size[2] ? 0 : 2) : (size[1] > size[2] ? 1 : 2);
            const float split = lo[axis] + size[axis] / 2.0f;  // midpoint of the node box, not of the centroids
            // two-pointer in-place partition; runs (and permutes) even when the node then stays a leaf
            int64_t i = first, j = int64_t(first) + int64_t(count) - 1;
            while (i <= j) {
                if (cen[3 * i + axis] < split) {
                    ++i;
                } else {
                    for (int k = 0; k < 3; ++k) {
                        std::swap(idx[3 * i + k], idx[3 * j + k]);
                        std::swap(cen[3 * i + k], cen[3 * j + k]);
                    }
                    --j;
                }
            }
            const uint32_t countA = uint32_t(i) - first, countB = count - countA;
            if (!(countA > 0 && countB > 0)) continue;    // split failed
            if (count <= kMaxNodeTriangleCount) continue;  // small enough
            const int32_t a = int32_t(nodes.size());
            UnityBounds ba = TriangleRangeBounds(first, countA, idx, V);
            nodes.push_back(MakeEntry(ba.Min(), ba.Max(), first, countA));
            if (countA > 2) next.push_back(a);
            const int32_t b = int32_t(nodes.size());
            UnityBounds bb = TriangleRangeBounds(uint32_t(i), countB, idx, V);
            nodes.push_back(MakeEntry(bb.Min(), bb.Max(), uint32_t(i), countB));
            if (countB > 2) next.push_back(b);
            cur.indexA = uint32_t(a);  // child B is always a + 1
            cur.triangleCount = 0;
            nodes[size_t(entry)] = cur;
        }
        queue.swap(next);
        next.clear();
    }
    const int64_t n = int64_t(nodes.size());
    if (out_nodes) {
        if (n > max_nodes) return -(n + 1);
        std::memcpy(out_nodes, nodes.data(), size_t(n) * sizeof(BVHEntry));
    }
    return n;
}

extern "C" int hg_pack_triangles(const float* V, const float* N, int32_t n_vertices, const int32_t* idx,
                                 int32_t n_tris, HalogenTriangle* out) {
    if (!V || !N || !idx || !out || n_tris < 0) return HG_E_INVALID;
    for (int64_t t = 0; t < n_tris; ++t) {
        int32_t i0 = idx[3 * t], i1 = idx[3 * t + 1], i2 = idx[3 * t + 2];
        if (i0 < 0 || i1 < 0 || i2 < 0 || i0 >= n_vertices || i1 >= n_vertices || i2 >= n_vertices)
            return HG_E_INVALID;
        HalogenTriangle& h = out[t];
        h.pointA = {V[3 * i0], V[3 * i0 + 1], V[3 * i0 + 2]};
        h.pointB = {V[3 * i1], V[3 * i1 + 1], V[3 * i1 + 2]};
        h.pointC = {V[3 * i2], V[3 * i2 + 1], V[3 * i2 + 2]};
        h.normalA = {N[3 * i0], N[3 * i0 + 1], N[3 * i0 + 2]};
        h.normalB = {N[3 * i1], N[3 * i1 + 1], N[3 * i1 + 2]};
        h.normalC = {N[3 * i2], N[3 * i2 + 1], N[3 * i2 + 2]};
    }
    return HG_OK;
}
