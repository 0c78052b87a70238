// tsan_blas — ThreadSanitizer driver of the parallel BLAS builder (hg_build_blas_mt, csrc/hg_host.cpp), built with
// g++ -fsanitize=thread straight from hg_host.cpp (make -C halogen-pathtracer_amd tsan; tests/test_sanitizers.py).
//
//   tsan_blas N_TRIS SEED THREADS...
// builds the BVH of a random triangle soup (N_TRIS >= 32,768 reaches the rank-parallel partition of large nodes)
// sequentially and with each thread count, and checks node arrays and reordered indices are identical.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "halogen_abi.h"

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s N_TRIS SEED THREADS...\n", argv[0]);
        return 2;
    }
    const int32_t n_tris = std::atoi(argv[1]);
    std::mt19937 rng(uint32_t(std::atoi(argv[2])));
    std::uniform_real_distribution<float> u(0.0f, 1.0f);
    std::vector<float> v(size_t(n_tris) * 9);
    float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
    for (int32_t t = 0; t < n_tris; ++t) {
        const float c[3] = {u(rng) * 10.0f, u(rng) * 4.0f, u(rng) * 10.0f};
        for (int k = 0; k < 3; ++k)
            for (int a = 0; a < 3; ++a) {
                float& p = v[(size_t(t) * 3 + k) * 3 + a];
                p = c[a] + u(rng) * 0.1f;
                lo[a] = p < lo[a] ? p : lo[a];
                hi[a] = p > hi[a] ? p : hi[a];
            }
    }
    std::vector<int32_t> idx0(size_t(n_tris) * 3);
    for (size_t i = 0; i < idx0.size(); ++i) idx0[i] = int32_t(i);
    const int64_t cap = 2 * int64_t(n_tris) + 1;
    std::vector<BVHEntry> ref(size_t(cap), BVHEntry{});
    std::vector<int32_t> ref_idx = idx0;
    const int64_t n_ref = hg_build_blas(v.data(), 3 * n_tris, ref_idx.data(), n_tris, lo, hi, 32, ref.data(), cap);
    if (n_ref <= 0) return 3;
    for (int a = 3; a < argc; ++a) {
        const int threads = std::atoi(argv[a]);
        std::vector<BVHEntry> got(size_t(cap), BVHEntry{});
        std::vector<int32_t> idx = idx0;
        const int64_t n = hg_build_blas_mt(v.data(), 3 * n_tris, idx.data(), n_tris, lo, hi, 32, got.data(), cap,
                                           threads);
        if (n != n_ref || std::memcmp(got.data(), ref.data(), size_t(n) * sizeof(BVHEntry)) != 0 || idx != ref_idx) {
            std::fprintf(stderr, "threads %d: parallel build differs from the sequential one\n", threads);
            return 4;
        }
        std::printf("threads %d: %lld entries, identical\n", threads, (long long)n);
    }
    return 0;
}
