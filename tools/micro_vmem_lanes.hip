// Microbenchmark: does a wave's 16-B-per-lane vector load cost the memory pipeline per instruction or per active
// lane?  Each wave runs `iters` dependent-free rounds of one global_load_dwordx4 per active lane from an L2-resident
// table (2 MiB), with 64 / 32 / 16 / 8 / 1 lanes active.  If the time per round falls with the active lanes, the
// texture path works per lane (partial waves in the relaxed descent cost only their lanes); if it stays flat, it
// works per instruction (a partial wave pays for 64 lanes).
//   hipcc --offload-arch=gfx950 -O3 tools/micro_vmem_lanes.hip -o tools/micro_vmem_lanes && tools/micro_vmem_lanes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(64) void loads(const float4* __restrict__ table, uint32_t mask_n, uint32_t iters,
                                            uint32_t table_f4, float* __restrict__ sink) {
    const uint32_t lane = threadIdx.x;
    float acc = 0.0f;
    if (lane < mask_n) {
        const uint32_t m = table_f4 - 1u;  // a power of two
        uint32_t idx = (blockIdx.x * 977u + lane * 131u) & m;
        for (uint32_t i = 0; i < iters; ++i) {
            const float4 v = table[idx];
            acc += v.x + v.y + v.z + v.w;
            idx = (idx + 4099u) & m;  // independent loads (throughput, not latency), each lane on its own line
        }
    }
    if (acc == 12345.0f) sink[blockIdx.x * 64u + lane] = acc;
}

// One traversal step's loads per lane: a 64-B node record (x4, x4, x3, x3 as the stream kernel issues them) at a
// random record, against only its first 16 B: how much do the extra requests to an already-fetched line cost?
template <int kLoads>
__global__ __launch_bounds__(64) void records(const float4* __restrict__ table, uint32_t iters, uint32_t table_f4,
                                              float* __restrict__ sink, uint32_t group) {
    const uint32_t lane = threadIdx.x;
    const uint32_t m = table_f4 / 4u - 1u;  // records of 4 float4
    // `group` consecutive lanes share a record (1: every lane its own line; 64: the whole wave on one record)
    uint32_t r = (blockIdx.x * 977u + (lane / group) * 131u) & m;
    float acc = 0.0f;
    for (uint32_t i = 0; i < iters; ++i) {
        const float4* p = table + 4u * r;
        const float4 a = p[0];
        acc += a.x + a.w;
        if (kLoads == 4) {
            const float4 b = p[1];
            const float3 c = *reinterpret_cast<const float3*>(p + 2), d = *reinterpret_cast<const float3*>(p + 3);
            acc += b.x + b.w + c.x + c.z + d.y;
        }
        r = (r + 1031u) & m;
    }
    if (acc == 12345.0f) sink[blockIdx.x * 64u + lane] = acc;
}

int main() {
    const uint32_t table_f4 = (2u << 20) / 16u, iters = 4096, blocks = 256 * 20 * 4;
    float4* table = nullptr;
    float* sink = nullptr;
    if (hipMalloc(&table, size_t(table_f4) * 16) != hipSuccess || hipMalloc(&sink, size_t(blocks) * 64 * 4) != hipSuccess)
        return 1;
    (void)hipMemset(table, 0, size_t(table_f4) * 16);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const uint32_t lanes[] = {64, 32, 16, 8, 1};
    for (uint32_t n : lanes) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(loads, dim3(blocks), dim3(64), 0, 0, table, n, iters, table_f4, sink);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        const double insts = double(blocks) * iters;
        printf("{\"active_lanes\": %u, \"ms\": %.3f, \"wave_loads_per_ns\": %.3f, \"lane_loads_per_ns\": %.3f}\n", n, best,
               insts / (best * 1e6), insts * n / (best * 1e6));
    }
    for (uint32_t group : {1u, 8u, 64u}) {
        for (int k : {1, 4}) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(a);
                if (k == 1)
                    hipLaunchKernelGGL(records<1>, dim3(blocks), dim3(64), 0, 0, table, iters, table_f4, sink, group);
                else
                    hipLaunchKernelGGL(records<4>, dim3(blocks), dim3(64), 0, 0, table, iters, table_f4, sink, group);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            const double recs = double(blocks) * iters * 64;
            printf("{\"lanes_per_record\": %u, \"record_loads_per_lane_step\": %d, \"ms\": %.3f, "
                   "\"lane_steps_per_ns\": %.3f}\n", group, k, best, recs / (best * 1e6));
        }
    }
    (void)hipFree(table);
    (void)hipFree(sink);
    return 0;
}
