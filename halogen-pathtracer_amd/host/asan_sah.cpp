// asan_sah — AddressSanitizer + UndefinedBehaviorSanitizer driver of the SAH BLAS builder (hg_build_blas_sah,
// csrc/hg_host.cpp), built with g++ -fsanitize=address,undefined straight from hg_host.cpp (make -C
// halogen-pathtracer_amd asan_sah; tests/test_sanitizers.py).
//
//   asan_sah N_TRIS SEED
// builds the SAH tree of a random triangle soup, of a flat grid (every box thin), of coincident triangles (every
// centroid equal), of denormal and near-FLT_MAX coordinates (a bin scale of inf or 0) and of an empty mesh, and checks
// every triangle lands in exactly one leaf; a NaN or infinite vertex is an invalid argument.
// Built with -fsanitize=float-cast-overflow too: no float -> int bin conversion may be out of range.
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <random>
#include <vector>

#include "halogen_abi.h"

static int check(const char* what, std::vector<float>& v, int32_t n_tris, int32_t max_leaf) {
    std::vector<int32_t> idx(size_t(n_tris) * 3 + 3);  // (never empty: a null list is an invalid argument)
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = int32_t(i % (v.size() / 3));
    const int64_t cap = 2 * int64_t(n_tris) + 2;
    std::vector<BVHEntry> nodes(static_cast<size_t>(cap));
    const int64_t n = hg_build_blas_sah(v.data(), int32_t(v.size() / 3), idx.data(), n_tris, max_leaf, 48, nodes.data(),
                                        cap);
    if (n <= 0) {
        std::fprintf(stderr, "%s: build failed %lld\n", what, (long long)n);
        return 3;
    }
    std::vector<int> seen(size_t(n_tris), 0);
    std::vector<int64_t> stack{0};
    int64_t reached = 0;
    while (!stack.empty()) {
        const int64_t g = stack.back();
        stack.pop_back();
        if (g < 0 || g >= n) return 4;
        ++reached;
        const BVHEntry& e = nodes[size_t(g)];
        if (e.triangleCount > 0) {
            for (uint32_t i = e.indexA; i < e.indexA + e.triangleCount; ++i) {
                if (i >= uint32_t(n_tris)) return 5;
                seen[i]++;
            }
        } else if (n_tris > 0) {
            stack.push_back(int64_t(e.indexA));
            stack.push_back(int64_t(e.indexA) + 1);
        }
    }
    for (int s : seen)
        if (s != 1) return 6;
    std::printf("%s: %d triangles, %lld entries, all reached (%lld), every triangle in one leaf\n", what, n_tris,
                (long long)n, (long long)reached);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s N_TRIS SEED\n", argv[0]);
        return 2;
    }
    const int32_t n_tris = std::atoi(argv[1]);
    std::mt19937 rng(uint32_t(std::atoi(argv[2])));
    std::uniform_real_distribution<float> u(0.0f, 1.0f);
    std::vector<float> soup(size_t(n_tris) * 9);
    for (int32_t t = 0; t < n_tris; ++t) {
        const float c[3] = {u(rng) * 10.0f, u(rng) * 4.0f, u(rng) * 10.0f};
        for (int k = 0; k < 9; ++k) soup[size_t(t) * 9 + k] = c[k % 3] + u(rng) * 0.1f;
    }
    std::vector<float> flat(size_t(n_tris) * 9);
    for (int32_t t = 0; t < n_tris; ++t)
        for (int k = 0; k < 3; ++k) {
            flat[size_t(t) * 9 + 3 * k] = float(t % 97) + float(k == 1);
            flat[size_t(t) * 9 + 3 * k + 1] = 0.0f;
            flat[size_t(t) * 9 + 3 * k + 2] = float(t / 97) + float(k == 2);
        }
    std::vector<float> same = {0, 0, 0, 1, 0, 0, 0, 1, 0};
    int rc = 0;
    for (int leaf : {1, 2, 4, 15}) {
        if ((rc = check("soup", soup, n_tris, leaf))) return rc;
        if ((rc = check("flat", flat, n_tris, leaf))) return rc;
    }
    if ((rc = check("coincident", same, 100, 2))) return rc;
    if ((rc = check("empty", same, 0, 2))) return rc;
    std::vector<float> tiny(soup), huge(soup);  // centroid spans of ~1e-38 (scale inf) and ~3e38 (extent inf)
    for (size_t i = 0; i < soup.size(); ++i) {
        tiny[i] = soup[i] * 1e-39f;
        huge[i] = (soup[i] - 5.0f) * 6e37f;
    }
    if ((rc = check("denormal", tiny, n_tris, 2))) return rc;
    if ((rc = check("huge", huge, n_tris, 2))) return rc;
    for (const float bad : {std::numeric_limits<float>::quiet_NaN(), std::numeric_limits<float>::infinity()}) {
        std::vector<float> v(soup);
        v[v.size() / 2] = bad;
        std::vector<int32_t> idx(size_t(n_tris) * 3 + 3);
        for (size_t i = 0; i < idx.size(); ++i) idx[i] = int32_t(i % (v.size() / 3));
        std::vector<BVHEntry> nodes(size_t(2 * n_tris + 2));
        const int64_t n = hg_build_blas_sah(v.data(), int32_t(v.size() / 3), idx.data(), n_tris, 2, 48, nodes.data(),
                                            int64_t(nodes.size()));
        if (n != HG_E_INVALID) {
            std::fprintf(stderr, "non-finite vertex: returned %lld\n", (long long)n);
            return 7;
        }
        std::printf("non-finite vertex rejected\n");
    }
    return 0;
}
