// Microbenchmark: what does a wave's vector load cost the texture-data path, per instruction or per byte returned?
// Each wave issues `iters` independent loads of 4 / 8 / 12 / 16 B per lane from an L2-resident table, with the 64
// lanes on 64 different 128-B lines (scattered) or on 4 lines (16 lanes per line, contiguous).  Reported per wave
// load instruction and per returned byte; DESIGN.md §10 uses it to price split or narrower record loads.
//   hipcc --offload-arch=gfx950 -O3 tools/micro_td_width.hip -o tools/micro_td_width && tools/micro_td_width
#include <hip/hip_runtime.h>

#include <cstdio>

template <int kDwords>
struct Vec;
template <> struct Vec<1> { typedef float T; };
template <> struct Vec<2> { typedef float2 T; };
template <> struct Vec<3> { typedef float3 T; };
template <> struct Vec<4> { typedef float4 T; };

__device__ __forceinline__ float sum(float v) { return v; }
__device__ __forceinline__ float sum(float2 v) { return v.x + v.y; }
__device__ __forceinline__ float sum(float3 v) { return v.x + v.y + v.z; }
__device__ __forceinline__ float sum(float4 v) { return v.x + v.y + v.z + v.w; }

template <int kDwords, bool kScatter>
__global__ __launch_bounds__(64) void loads(const float* __restrict__ table, uint32_t iters, uint32_t lines,
                                            float* __restrict__ sink) {
    typedef typename Vec<kDwords>::T T;
    const uint32_t lane = threadIdx.x;
    // 128-B line index per lane: scattered = own line; contiguous = 16 lanes share a line (4 lines per wave)
    uint32_t line = (blockIdx.x * 977u + (kScatter ? lane * 131u : (lane >> 4) * 131u)) & (lines - 1u);
    const uint32_t within = kScatter ? 0u : (lane & 15u) * 8u;  // byte offset / 4 inside the line (8 B apart ... )
    float acc = 0.0f;
    for (uint32_t i = 0; i < iters; ++i) {
        const T v = *reinterpret_cast<const T*>(table + line * 32u + (within & (32u - kDwords)));
        acc += sum(v);
        line = (line + 4099u) & (lines - 1u);
    }
    if (acc == 12345.0f) sink[blockIdx.x * 64u + lane] = acc;
}

template <int kDwords, bool kScatter>
float run(const float* table, uint32_t iters, uint32_t lines, float* sink, uint32_t blocks, hipEvent_t a, hipEvent_t b) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((loads<kDwords, kScatter>), dim3(blocks), dim3(64), 0, 0, table, iters, lines, sink);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best;
}

int main() {
    const uint32_t lines = (2u << 20) / 128u, iters = 4096, blocks = 256 * 20 * 4;
    float* table = nullptr;
    float* sink = nullptr;
    if (hipMalloc(&table, size_t(lines) * 128) != hipSuccess || hipMalloc(&sink, size_t(blocks) * 64 * 4) != hipSuccess)
        return 1;
    (void)hipMemset(table, 0, size_t(lines) * 128);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const double insts = double(blocks) * iters;
    float ms[2][4];
    ms[0][0] = run<1, true>(table, iters, lines, sink, blocks, a, b);
    ms[0][1] = run<2, true>(table, iters, lines, sink, blocks, a, b);
    ms[0][2] = run<3, true>(table, iters, lines, sink, blocks, a, b);
    ms[0][3] = run<4, true>(table, iters, lines, sink, blocks, a, b);
    ms[1][0] = run<1, false>(table, iters, lines, sink, blocks, a, b);
    ms[1][1] = run<2, false>(table, iters, lines, sink, blocks, a, b);
    ms[1][2] = run<3, false>(table, iters, lines, sink, blocks, a, b);
    ms[1][3] = run<4, false>(table, iters, lines, sink, blocks, a, b);
    for (int s = 0; s < 2; ++s)
        for (int w = 0; w < 4; ++w)
            printf("{\"lanes\": \"%s\", \"bytes_per_lane\": %d, \"ms\": %.3f, \"wave_loads_per_ns\": %.3f, "
                   "\"gpu_cycles_per_wave_load_per_cu\": %.2f, \"bytes_per_ns\": %.1f}\n",
                   s == 0 ? "64 lines" : "4 lines", 4 * (w + 1), ms[s][w], insts / (ms[s][w] * 1e6),
                   ms[s][w] * 1e-3 * 2.4e9 * 256.0 / insts, insts * 64.0 * 4 * (w + 1) / (ms[s][w] * 1e6));
    (void)hipFree(table);
    (void)hipFree(sink);
    return 0;
}
