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
#include <atomic>
#include <cfloat>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <cstring>
#include <limits>
#include <thread>
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

// ---------------------------------------------------------------------------------------------------
// Parallel build (hg_build_blas_mt): the same node array and the same reordered triangle list as hg_build_blas,
// level by level.  Within a BFS level the queue entries own disjoint triangle ranges, so they are independent:
// small entries run the sequential partition + bounds on a worker each, large ones use all workers:
//  - bounds: chunked folds of `a < b ? a : b` / `a > b ? a : b`, combined in range order.  Without NaN that fold
//    is associative (it keeps the LAST occurrence of the extreme, so +0/-0 ties resolve as sequentially); a
//    vertex array holding a NaN makes the whole build sequential.
//  - partition: the two-pointer loop above moves elements by a rule that depends only on ranks.  With A the
//    number of left (cen < split) elements, p_1 < .. < p_r the right elements in [0, A), q_1 > .. > q_r the left
//    elements in [A, n) and q_0 = n:  left x < A stays;  p_k -> q_{k-1} - 1;  q_k -> p_k;  a right x > A -> x - 1;
//    a right x == A -> q_r - 1.  (Derived from the loop; tests/test_bvh.py checks it against the sequential build.)
// Node numbering follows the queue order, so it is assigned sequentially after each level.
// ---------------------------------------------------------------------------------------------------
namespace {

// A fixed set of workers for one build: run(f) calls f(t) on every worker t in [0, n) and returns when all are done
// (the calling thread is worker 0).  Starting threads once per build, not once per pass, keeps the per-pass cost
// at a wake-up.
class Workers {
  public:
    explicit Workers(int n) : n_(n) {
        for (int t = 1; t < n_; ++t) pool_.emplace_back([this, t] { loop(t); });
    }
    ~Workers() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& th : pool_) th.join();
    }
    int size() const { return n_; }
    template <class F>
    void run(F&& f) {
        if (n_ == 1) {
            f(0);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            task_ = std::function<void(int)>(std::forward<F>(f));
            pending_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        task_(0);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return pending_ == 0; });
    }
    // f(t, lo, hi) over n_ contiguous chunks of [0, n)
    template <class F>
    void chunks(int64_t n, F&& f) {
        run([&](int t) { f(t, n * t / n_, n * (t + 1) / n_); });
    }

  private:
    void loop(int t) {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> g(m_);
            cv_.wait(g, [&] { return gen_ != seen; });
            seen = gen_;
            if (stop_) return;
            g.unlock();
            task_(t);
            g.lock();
            if (--pending_ == 0) done_.notify_one();
        }
    }
    int n_;
    std::vector<std::thread> pool_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    std::function<void(int)> task_;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};

struct Box {
    Vec3 mn, mx;
};

Box fold_range(uint64_t lo, uint64_t hi, const int32_t* idx, const float* V) {
    const float inf = std::numeric_limits<float>::infinity();
    Box b{{{inf, inf, inf}}, {{-inf, -inf, -inf}}};
    for (uint64_t i = lo; i < hi; ++i)
        for (int c = 0; c < 3; ++c) {
            const float* p = V + 3 * int64_t(idx[3 * i + c]);
            for (int k = 0; k < 3; ++k) {
                b.mn[k] = b.mn[k] < p[k] ? b.mn[k] : p[k];
                b.mx[k] = b.mx[k] > p[k] ? b.mx[k] : p[k];
            }
        }
    return b;
}

UnityBounds range_bounds_mt(uint32_t start, uint32_t count, const int32_t* idx, const float* V, Workers& w) {
    std::vector<Box> part(size_t(w.size()));
    w.chunks(count, [&](int t, int64_t lo, int64_t hi) {
        part[size_t(t)] = fold_range(uint64_t(start) + lo, uint64_t(start) + hi, idx, V);
    });
    Box b = part[0];
    for (size_t t = 1; t < part.size(); ++t)  // combine in range order, same rule as the fold
        for (int k = 0; k < 3; ++k) {
            b.mn[k] = b.mn[k] < part[t].mn[k] ? b.mn[k] : part[t].mn[k];
            b.mx[k] = b.mx[k] > part[t].mx[k] ? b.mx[k] : part[t].mx[k];
        }
    UnityBounds u = UnityBounds::FromMinMax(b.mn, b.mx);
    u.PadIfThin();
    return u;
}

// The sequential two-pointer partition of [first, first+count) (hg_build_blas), returning the left count.
uint32_t partition_seq(uint32_t first, uint32_t count, int axis, float split, int32_t* idx, float* cen) {
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
    return uint32_t(i - first);
}

// The same permutation computed from ranks (rule above) by every worker; tmp_*, P and Q hold `count` entries.
uint32_t partition_mt(uint32_t first, uint32_t count, int axis, float split, int32_t* idx, float* cen,
                      std::vector<int32_t>& tmp_i, std::vector<float>& tmp_c, std::vector<uint32_t>& P,
                      std::vector<uint32_t>& Q, Workers& w) {
    const int64_t n = count;
    const int T = w.size();
    int32_t* I = idx + 3 * int64_t(first);
    float* Cn = cen + 3 * int64_t(first);
    std::vector<int64_t> cntL(size_t(T) + 1, 0), frontL(size_t(T), 0);
    w.chunks(n, [&](int t, int64_t lo, int64_t hi) {
        int64_t c = 0;
        for (int64_t x = lo; x < hi; ++x) c += Cn[3 * x + axis] < split;
        cntL[size_t(t) + 1] = c;
    });
    for (int t = 0; t < T; ++t) cntL[size_t(t) + 1] += cntL[size_t(t)];  // left elements before each chunk
    const int64_t A = cntL[size_t(T)];
    if (P.size() < size_t(n)) {
        P.resize(size_t(n));
        Q.resize(size_t(n));
        tmp_i.resize(size_t(3 * n));
        tmp_c.resize(size_t(3 * n));
    }
    // P[k-1] = p_k, the k-th right element in [0, A); Q[k-1] = q_k, the k-th left element in [A, n) from the end
    w.chunks(n, [&](int t, int64_t lo, int64_t hi) {
        int64_t pl = cntL[size_t(t)], fl = 0;  // left elements in [0, x); left elements of this chunk below A
        for (int64_t x = lo; x < hi; ++x) {
            const bool left = Cn[3 * x + axis] < split;
            if (x < A) {
                if (left) ++fl;
                else P[size_t(x - pl)] = uint32_t(x);  // rank - 1 = rights in [0, x)
            } else if (left) {
                Q[size_t(A - pl - 1)] = uint32_t(x);  // rank = lefts in [x, n)
            }
            pl += left;
        }
        frontL[size_t(t)] = fl;
    });
    int64_t r = A;  // right elements in [0, A)
    for (int t = 0; t < T; ++t) r -= frontL[size_t(t)];
    const int64_t qr_minus_1 = (r == 0 ? n : int64_t(Q[size_t(r - 1)])) - 1;
    w.chunks(n, [&](int t, int64_t lo, int64_t hi) {
        int64_t pl = cntL[size_t(t)];
        for (int64_t x = lo; x < hi; ++x) {
            const bool left = Cn[3 * x + axis] < split;
            int64_t dst;
            if (x < A) {
                if (left) {
                    dst = x;
                } else {
                    const int64_t k = (x + 1) - pl;  // p_k -> q_{k-1} - 1
                    dst = (k == 1 ? n : int64_t(Q[size_t(k - 2)])) - 1;
                }
            } else if (left) {
                dst = P[size_t(A - pl - 1)];  // q_k -> p_k
            } else {
                dst = x == A ? qr_minus_1 : x - 1;
            }
            for (int c = 0; c < 3; ++c) {
                tmp_i[size_t(3 * dst + c)] = I[3 * x + c];
                tmp_c[size_t(3 * dst + c)] = Cn[3 * x + c];
            }
            pl += left;
        }
    });
    w.chunks(n, [&](int, int64_t lo, int64_t hi) {
        std::memcpy(I + 3 * lo, tmp_i.data() + 3 * lo, size_t(3 * (hi - lo)) * sizeof(int32_t));
        std::memcpy(Cn + 3 * lo, tmp_c.data() + 3 * lo, size_t(3 * (hi - lo)) * sizeof(float));
    });
    return uint32_t(A);
}

struct LevelResult {
    uint32_t countA;
    bool split;
    UnityBounds ba, bb;
};

}  // namespace

extern "C" int64_t hg_build_blas_mt(const float* V, int32_t n_vertices, int32_t* idx, int32_t n_tris,
                                    const float root_min[3], const float root_max[3], int32_t max_hierarchy_depth,
                                    BVHEntry* out_nodes, int64_t max_nodes, int32_t n_threads) {
    if (!V || !idx || n_tris < 0 || n_vertices < 0 || !root_min || !root_max) return HG_E_INVALID;
    for (int64_t i = 0; i < 3 * int64_t(n_tris); ++i)
        if (idx[i] < 0 || idx[i] >= n_vertices) return HG_E_INVALID;
    int threads = n_threads > 0 ? n_threads : int(std::thread::hardware_concurrency());
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    for (int64_t i = 0; i < 3 * int64_t(n_vertices); ++i)
        if (V[i] != V[i]) return hg_build_blas(V, n_vertices, idx, n_tris, root_min, root_max, max_hierarchy_depth,
                                               out_nodes, max_nodes);  // NaN: order-exact sequential build
    if (threads == 1 || n_tris < 4096)
        return hg_build_blas(V, n_vertices, idx, n_tris, root_min, root_max, max_hierarchy_depth, out_nodes,
                             max_nodes);

    std::vector<BVHEntry> nodes;
    nodes.reserve(size_t(2) * size_t(n_tris) + 1);
    {
        UnityBounds rb = UnityBounds::FromMinMax(Vec3{{root_min[0], root_min[1], root_min[2]}},
                                                 Vec3{{root_max[0], root_max[1], root_max[2]}});
        nodes.push_back(MakeEntry(rb.Min(), rb.Max(), 0, uint32_t(n_tris)));
    }
    Workers w(threads);
    std::vector<float> cen(size_t(n_tris) * 3);
    w.chunks(n_tris, [&](int, int64_t lo, int64_t hi) {
        for (int64_t t = lo; t < hi; ++t) {
            const float* a = V + 3 * int64_t(idx[3 * t]);
            const float* b = V + 3 * int64_t(idx[3 * t + 1]);
            const float* c = V + 3 * int64_t(idx[3 * t + 2]);
            for (int k = 0; k < 3; ++k) cen[size_t(3 * t + k)] = ((a[k] + b[k]) + c[k]) / 3.0f;
        }
    });
    constexpr uint32_t kBig = 1u << 15;  // entries this large use every worker
    std::vector<int32_t> tmp_i;
    std::vector<float> tmp_c;
    std::vector<uint32_t> P, Q;
    std::vector<int32_t> queue{0}, next;
    std::vector<LevelResult> res;
    for (int depth = 1; depth <= max_hierarchy_depth && !queue.empty(); ++depth) {
        res.assign(queue.size(), LevelResult{0, false, {}, {}});
        auto node_geometry = [&](const BVHEntry& cur, int& axis, float& split) {
            const float size[3] = {cur.boundingCornerB.x - cur.boundingCornerA.x,
                                   cur.boundingCornerB.y - cur.boundingCornerA.y,
                                   cur.boundingCornerB.z - cur.boundingCornerA.z};
            const float lo[3] = {cur.boundingCornerA.x, cur.boundingCornerA.y, cur.boundingCornerA.z};
            axis = size[0] > size[1] ? (size[0] > size[2] ? 0 : 2) : (size[1] > size[2] ? 1 : 2);
            split = lo[axis] + size[axis] / 2.0f;
        };
        // large entries, one at a time with every worker
        for (size_t q = 0; q < queue.size(); ++q) {
            const BVHEntry& cur = nodes[size_t(queue[q])];
            if (cur.triangleCount < kBig) continue;
            int axis;
            float split;
            node_geometry(cur, axis, split);
            const uint32_t first = cur.indexA, count = cur.triangleCount;
            const uint32_t countA = partition_mt(first, count, axis, split, idx, cen.data(), tmp_i, tmp_c, P, Q, w);
            LevelResult& r = res[q];
            r.countA = countA;
            r.split = countA > 0 && count - countA > 0 && count > kMaxNodeTriangleCount;
            if (r.split) {
                r.ba = range_bounds_mt(first, countA, idx, V, w);
                r.bb = range_bounds_mt(first + countA, count - countA, idx, V, w);
            }
        }
        // small entries, spread over the workers in blocks of 32 (dynamic: sizes differ)
        std::atomic<size_t> cursor{0};
        constexpr size_t kBlock = 32;
        auto small = [&](int) {
            for (;;) {
                const size_t q0 = cursor.fetch_add(kBlock);
                if (q0 >= queue.size()) break;
                for (size_t q = q0; q < q0 + kBlock && q < queue.size(); ++q) {
                const BVHEntry& cur = nodes[size_t(queue[q])];
                if (cur.triangleCount >= kBig) continue;
                int axis;
                float split;
                node_geometry(cur, axis, split);
                const uint32_t first = cur.indexA, count = cur.triangleCount;
                const uint32_t countA = partition_seq(first, count, axis, split, idx, cen.data());
                LevelResult& r = res[q];
                r.countA = countA;
                r.split = countA > 0 && count - countA > 0 && count > kMaxNodeTriangleCount;
                if (r.split) {
                    r.ba = TriangleRangeBounds(first, countA, idx, V);
                    r.bb = TriangleRangeBounds(first + countA, count - countA, idx, V);
                }
                }
            }
        };
        if (queue.size() > 64) w.run(small);
        else small(0);
        // numbering in queue order (BVHGenerator.cs:40-129)
        for (size_t q = 0; q < queue.size(); ++q) {
            if (!res[q].split) continue;
            BVHEntry cur = nodes[size_t(queue[q])];
            const uint32_t first = cur.indexA, count = cur.triangleCount, countA = res[q].countA;
            const int32_t a = int32_t(nodes.size());
            nodes.push_back(MakeEntry(res[q].ba.Min(), res[q].ba.Max(), first, countA));
            if (countA > 2) next.push_back(a);
            nodes.push_back(MakeEntry(res[q].bb.Min(), res[q].bb.Max(), first + countA, count - countA));
            if (count - countA > 2) next.push_back(a + 1);
            cur.indexA = uint32_t(a);
            cur.triangleCount = 0;
            nodes[size_t(queue[q])] = cur;
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

// ---------------------------------------------------------------------------------------------------------------------
// Fast BLAS ("an SAH variant behind a non-parity flag"): a binned surface-area-heuristic build
// that emits the reference's BVHEntry format — children of entry g at indexA and indexA + 1, leaves holding a range of
// the reordered triangle list — so hg_upload_scene, the traversal and the CPU oracle take it unchanged.  Its images are
// those of a different (valid) hierarchy, not the reference builder's: rays find the same nearest triangle except
// where two lie within rounding of each other, and every traversal counter differs.  The GPU render of an SAH
// hierarchy is still bit-exact against the oracle's render of the same hierarchy (tests/test_gpu_fast_bvh.py).
// Boxes are their triangles' float min / max through the reference's Bounds arithmetic (padded when thin).
// ---------------------------------------------------------------------------------------------------------------------
namespace {

struct Box3 {
    float lo[3] = {std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(),
                   std::numeric_limits<float>::infinity()};
    float hi[3] = {-std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                   -std::numeric_limits<float>::infinity()};
    void add(const float* p) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = p[k] < lo[k] ? p[k] : lo[k];
            hi[k] = p[k] > hi[k] ? p[k] : hi[k];
        }
    }
    void add(const Box3& b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = b.lo[k] < lo[k] ? b.lo[k] : lo[k];
            hi[k] = b.hi[k] > hi[k] ? b.hi[k] : hi[k];
        }
    }
    double area() const {
        if (!(hi[0] >= lo[0])) return 0.0;
        const double dx = double(hi[0]) - lo[0], dy = double(hi[1]) - lo[1], dz = double(hi[2]) - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

constexpr int kSahBins = 32;

// The bin of a centroid coordinate: computed and clamped in float, so that no float -> int conversion is out of range
// (a centroid span of a few ulps gives a scale near FLT_MAX, and (c - lo) * scale may then overflow to inf)
inline int sah_bin(float c, float lo, float scale) {
    const float f = (c - lo) * scale;
    if (!(f > 0.0f)) return 0;
    if (!(f < float(kSahBins - 1))) return kSahBins - 1;
    return int(f);
}

}  // namespace

extern "C" int64_t hg_build_blas_sah(const float* V, int32_t n_vertices, int32_t* idx, int32_t n_tris,
                                     int32_t max_leaf, int32_t max_depth, BVHEntry* out_nodes, int64_t max_nodes) {
    if (!V || !idx || n_tris < 0 || n_vertices < 0 || max_leaf < 1 || max_leaf > 15 || max_depth < 1) return HG_E_INVALID;
    for (int64_t i = 0; i < 3 * int64_t(n_tris); ++i) {
        if (idx[i] < 0 || idx[i] >= n_vertices) return HG_E_INVALID;
        const float* p = V + 3 * size_t(idx[i]);  // a NaN or infinite vertex has no box (and no bin)
        if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) return HG_E_INVALID;
    }
    const size_t n = size_t(n_tris);
    std::vector<Box3> tb(n);
    std::vector<float> cen(3 * n);
    for (size_t t = 0; t < n; ++t) {
        for (int v = 0; v < 3; ++v) tb[t].add(V + 3 * size_t(idx[3 * t + v]));
        for (int k = 0; k < 3; ++k) cen[3 * t + k] = 0.5f * tb[t].lo[k] + 0.5f * tb[t].hi[k];
    }
    std::vector<uint32_t> ord(n);  // triangle order; idx is rewritten from it at the end
    for (size_t t = 0; t < n; ++t) ord[t] = uint32_t(t);
    std::vector<BVHEntry> nodes;
    nodes.reserve(2 * n + 1);
    // boxes through the reference's Bounds arithmetic (centre / extents round trip, and the AABBEpsilon pad of a box
    // thinner than it on any axis, BVHGenerator.cs:154-186): a flat wall's leaves keep the thickness every traversal
    // of the reference relies on
    auto entry = [&](uint32_t first, uint32_t count, const Box3& b) {
        UnityBounds u = UnityBounds::FromMinMax(Vec3{{b.lo[0], b.lo[1], b.lo[2]}}, Vec3{{b.hi[0], b.hi[1], b.hi[2]}});
        u.PadIfThin();
        return MakeEntry(u.Min(), u.Max(), first, count);
    };
    auto range_box = [&](uint32_t first, uint32_t count) {
        Box3 b;
        for (uint32_t i = first; i < first + count; ++i) b.add(tb[ord[i]]);
        return b;
    };
    nodes.push_back(entry(0, uint32_t(n), range_box(0, uint32_t(n))));
    if (n == 0) nodes[0].triangleCount = 0, nodes[0].indexA = 0;
    struct Job {
        uint32_t node, depth;
    };
    std::vector<Job> jobs{{0u, 0u}};
    while (!jobs.empty()) {
        const Job j = jobs.back();
        jobs.pop_back();
        const uint32_t first = nodes[j.node].indexA, count = nodes[j.node].triangleCount;
        if (count <= uint32_t(max_leaf) || j.depth + 1 >= uint32_t(max_depth)) {
            if (count > 15u && j.depth + 1 >= uint32_t(max_depth)) return HG_E_UNSUPPORTED;  // too deep to split
            continue;
        }
        Box3 cb;  // centroid bounds
        for (uint32_t i = first; i < first + count; ++i) cb.add(&cen[3 * size_t(ord[i])]);
        int best_axis = -1;
        uint32_t best_bin = 0;
        double best_cost = std::numeric_limits<double>::infinity();
        for (int ax = 0; ax < 3; ++ax) {
            const float ext = cb.hi[ax] - cb.lo[ax];
            const float scale = float(kSahBins) / ext;
            if (!(ext > 0.0f) || !(scale < FLT_MAX)) continue;  // one centroid plane (or a span of denormals)
            Box3 bins[kSahBins];
            uint32_t cnt[kSahBins] = {};
            for (uint32_t i = first; i < first + count; ++i) {
                const uint32_t t = ord[i];
                const int b = sah_bin(cen[3 * size_t(t) + ax], cb.lo[ax], scale);
                bins[b].add(tb[t]);
                cnt[b]++;
            }
            double right_area[kSahBins];
            uint32_t right_cnt[kSahBins];
            Box3 acc;
            uint32_t c = 0;
            for (int b = kSahBins - 1; b > 0; --b) {
                acc.add(bins[b]);
                c += cnt[b];
                right_area[b] = acc.area();
                right_cnt[b] = c;
            }
            Box3 left;
            uint32_t lc = 0;
            for (int b = 0; b < kSahBins - 1; ++b) {
                left.add(bins[b]);
                lc += cnt[b];
                if (lc == 0 || right_cnt[b + 1] == 0) continue;
                const double cost = left.area() * lc + right_area[b + 1] * right_cnt[b + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = ax;
                    best_bin = uint32_t(b);
                }
            }
        }
        const double parent_area = nodes[j.node].triangleCount ? range_box(first, count).area() : 0.0;
        // leaf if no split separates the centroids, or (small enough to be an inline leaf) splitting costs more than
        // testing every triangle (traversal step ~ one triangle test)
        uint32_t mid = first;
        if (best_axis >= 0) {
            const float ext = cb.hi[best_axis] - cb.lo[best_axis], scale = float(kSahBins) / ext;
            uint32_t* lo = ord.data() + first;
            uint32_t* hi = ord.data() + first + count;
            while (lo < hi) {
                const int b = sah_bin(cen[3 * size_t(*lo) + best_axis], cb.lo[best_axis], scale);
                if (uint32_t(b) <= best_bin) ++lo;
                else std::swap(*lo, *--hi);
            }
            mid = uint32_t(lo - ord.data());
            if (count <= 15u && parent_area > 0.0 && 1.0 + best_cost / parent_area >= double(count)) continue;
        }
        if (mid == first || mid == first + count) {  // degenerate centroids: split the range in half
            if (count <= 15u) continue;
            mid = first + count / 2;
        }
        const uint32_t a = uint32_t(nodes.size());
        nodes.push_back(entry(first, mid - first, range_box(first, mid - first)));
        nodes.push_back(entry(mid, first + count - mid, range_box(mid, first + count - mid)));
        nodes[j.node].indexA = a;
        nodes[j.node].triangleCount = 0;
        jobs.push_back({a + 1, j.depth + 1});
        jobs.push_back({a, j.depth + 1});
    }
    std::vector<int32_t> re(3 * n);
    for (size_t i = 0; i < n; ++i)
        for (int v = 0; v < 3; ++v) re[3 * i + v] = idx[3 * size_t(ord[i]) + v];
    if (!re.empty()) std::memcpy(idx, re.data(), re.size() * sizeof(int32_t));
    const int64_t nn = int64_t(nodes.size());
    if (out_nodes) {
        if (nn > max_nodes) return -(nn + 1);
        std::memcpy(out_nodes, nodes.data(), size_t(nn) * sizeof(BVHEntry));
    }
    return nn;
}
