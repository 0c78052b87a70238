// Microbenchmark for the ray-coherence lever (DESIGN.md §10 lever 7): does the ORDER of a wave's
// lanes change what a vector load costs the texture-data path, for a fixed set of cache lines per instruction?
// Each wave issues `iters` independent 16-B loads from an L2-resident table; per instruction its 64 lanes fall on L
// distinct 128-B lines (lanes on one line read the same 16 B, as traversal lanes at one node read one record).  Lanes
// are mapped to the L lines
//   grouped      lane i -> line i * L / 64 (a line's lanes adjacent: what sorting the rays by octant would produce)
//   interleaved  lane i -> line i % L      (a line's lanes spread across the wave)
//   shuffled     lane i -> line perm(i) * L / 64 (a fixed random permutation of the grouped map)
// If the three cost the same for every L, re-ordering rays among a wave's lanes cannot relieve the TD unit: only the
// number of distinct lines per instruction (which rays share a wave) matters.
//   hipcc --offload-arch=gfx950 -O3 tools/micro_lane_order.hip -o tools/micro_lane_order && tools/micro_lane_order
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(64) void loads(const float4* __restrict__ table, uint32_t iters, uint32_t lines,
                                            const uint32_t* __restrict__ lane_line, float* __restrict__ sink) {
    const uint32_t lane = threadIdx.x;
    uint32_t line = (blockIdx.x * 977u + lane_line[lane] * 131u) & (lines - 1u);
    float acc = 0.0f;
    for (uint32_t i = 0; i < iters; ++i) {
        const float4 v = table[line * 8u];  // 8 float4 per 128-B line: the line's first 16 B
        acc += v.x + v.y + v.z + v.w;
        line = (line + 4099u) & (lines - 1u);
    }
    if (acc == 12345.0f) sink[blockIdx.x * 64u + lane] = acc;
}

int main() {
    const uint32_t lines = (2u << 20) / 128u, iters = 4096, blocks = 256 * 20 * 4;
    float4* table = nullptr;
    float* sink = nullptr;
    uint32_t* map = nullptr;
    if (hipMalloc(&table, size_t(lines) * 128) != hipSuccess || hipMalloc(&sink, size_t(blocks) * 64 * 4) != hipSuccess ||
        hipMalloc(&map, 64 * sizeof(uint32_t)) != hipSuccess)
        return 1;
    (void)hipMemset(table, 0, size_t(lines) * 128);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    uint32_t perm[64];
    for (uint32_t i = 0; i < 64; ++i) perm[i] = i;
    uint32_t x = 12345u;
    for (uint32_t i = 63; i > 0; --i) {  // Fisher-Yates with an LCG
        x = x * 1664525u + 1013904223u;
        const uint32_t j = (x >> 8) % (i + 1);
        const uint32_t t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
    const double insts = double(blocks) * iters;
    const char* names[3] = {"grouped", "interleaved", "shuffled"};
    for (uint32_t L : {1u, 2u, 4u, 8u, 16u, 32u, 64u}) {
        for (int mode = 0; mode < 3; ++mode) {
            uint32_t h[64];
            for (uint32_t i = 0; i < 64; ++i)
                h[i] = mode == 0 ? i * L / 64u : mode == 1 ? i % L : perm[i] * L / 64u;
            (void)hipMemcpy(map, h, sizeof h, hipMemcpyHostToDevice);
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(a);
                hipLaunchKernelGGL(loads, dim3(blocks), dim3(64), 0, 0, table, iters, lines, map, sink);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            printf("{\"lines_per_inst\": %u, \"lane_map\": \"%s\", \"ms\": %.3f, \"wave_loads_per_ns\": %.3f, "
                   "\"gpu_cycles_per_wave_load_per_cu\": %.2f}\n",
                   L, names[mode], best, insts / (best * 1e6), best * 1e-3 * 2.4e9 * 256.0 / insts);
        }
    }
    (void)hipFree(table);
    (void)hipFree(sink);
    (void)hipFree(map);
    return 0;
}
