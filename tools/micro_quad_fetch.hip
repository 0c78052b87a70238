// Microbenchmark for DESIGN.md §10 lever 4 (quad-cooperative node fetch): a traversal step loads one 64-B record per
// lane with four 16-B loads, so every wave load instruction touches up to 64 records.  Cooperatively, the four lanes
// of a quad fetch the quad's four records one after another (round j: lane q loads quarter q of quad-lane j's record,
// so an instruction touches 16 records, each as one contiguous 64 B), then a 4x4 transpose inside the quad (two DPP
// butterfly stages) hands each lane its own record.  Same records, same sums; compares time per lane-step.
//   hipcc --offload-arch=gfx950 -O3 tools/micro_quad_fetch.hip -o tools/micro_quad_fetch && tools/micro_quad_fetch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ __forceinline__ float dpp_xor1(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));  // quad_perm 1,0,3,2
}
__device__ __forceinline__ float dpp_xor2(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));  // quad_perm 2,3,0,1
}
__device__ __forceinline__ uint32_t dpp_bcast(uint32_t v, int j) {  // quad lane j's value to the whole quad
    switch (j) {
        case 0: return uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0x00, 0xF, 0xF, false));
        case 1: return uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0x55, 0xF, 0xF, false));
        case 2: return uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0xAA, 0xF, 0xF, false));
        default: return uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0xFF, 0xF, 0xF, false));
    }
}

// One butterfly stage over the float4 columns (a, b) = (j, j ^ s), bit s of j clear: the lane with bit s of q clear
// takes its partner's column a into its column b, the other lane takes its partner's column b into its column a.
// As selects of partner values: a' = hi ? partner.b : a, b' = hi ? b : partner.a (a DPP-sourced v_cndmask each).
template <int S>
__device__ __forceinline__ float xs(float v) { return S == 1 ? dpp_xor1(v) : dpp_xor2(v); }
template <int S>
__device__ __forceinline__ void stage(float4& a, float4& b, bool hi) {
    const float4 pa = make_float4(xs<S>(a.x), xs<S>(a.y), xs<S>(a.z), xs<S>(a.w));  // partner's a, b
    const float4 pb = make_float4(xs<S>(b.x), xs<S>(b.y), xs<S>(b.z), xs<S>(b.w));
    a = make_float4(hi ? pb.x : a.x, hi ? pb.y : a.y, hi ? pb.z : a.z,
                    hi ? pb.w : a.w);
    b = make_float4(hi ? b.x : pa.x, hi ? b.y : pa.y, hi ? b.z : pa.z, hi ? b.w : pa.w);
}

template <bool kQuad>
__global__ __launch_bounds__(64) void records(const float4* __restrict__ table, uint32_t iters, uint32_t table_f4,
                                              float* __restrict__ sink, uint32_t group) {
    const uint32_t lane = threadIdx.x, q = lane & 3u;
    const uint32_t m = table_f4 / 4u - 1u;  // records of 4 float4
    uint32_t r = (blockIdx.x * 977u + (lane / group) * 131u) & m;
    float acc = 0.0f;
    for (uint32_t i = 0; i < iters; ++i) {
        float4 c0, c1, c2, c3;  // this lane's record, quarters 0..3
        if (kQuad) {
            // round j: quarter q of quad-lane j's record -> column j
            float4 R0 = table[4u * dpp_bcast(r, 0) + q];
            float4 R1 = table[4u * dpp_bcast(r, 1) + q];
            float4 R2 = table[4u * dpp_bcast(r, 2) + q];
            float4 R3 = table[4u * dpp_bcast(r, 3) + q];
            stage<1>(R0, R1, (q & 1u) != 0u);
            stage<1>(R2, R3, (q & 1u) != 0u);
            stage<2>(R0, R2, (q & 2u) != 0u);
            stage<2>(R1, R3, (q & 2u) != 0u);
            c0 = R0; c1 = R1; c2 = R2; c3 = R3;
        } else {
            const float4* p = table + 4u * r;
            c0 = p[0]; c1 = p[1]; c2 = p[2]; c3 = p[3];
        }
        acc += c0.x + c0.y + c0.z + c0.w + c1.x + c1.y + c1.z + c1.w + c2.x + c2.y + c2.z + c3.x + c3.y + c3.z;
        r = (r + 1031u) & m;
    }
    sink[blockIdx.x * 64u + lane] = acc;
}

// The same cooperative rounds through LDS: round j's loads go straight into LDS (gfx950's 16-B global_load_lds),
// lane l's 16 B at slot j * 64 + l, so quad-lane j's whole record lands at slots 4k+0..3 of round j's kilobyte; each lane
// then reads its record back with four 16-B LDS reads.  No transpose VALU; 4 KB of LDS per wave.
__global__ __launch_bounds__(64) void records_lds(const float4* __restrict__ table, uint32_t iters, uint32_t table_f4,
                                                  float* __restrict__ sink, uint32_t group) {
    __shared__ float4 stage_lds[4 * 64];
    const uint32_t lane = threadIdx.x, q = lane & 3u, j_own = lane & 3u, quad = lane & ~3u;
    const uint32_t m = table_f4 / 4u - 1u;
    uint32_t r = (blockIdx.x * 977u + (lane / group) * 131u) & m;
    float acc = 0.0f;
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t rj = dpp_bcast(r, int(j));
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(table + 4u * rj + q),
                (__attribute__((address_space(3))) void*)(stage_lds + j * 64u), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const float4* mine = stage_lds + j_own * 64u + quad;  // round j_own, slots quad+0..3
        const float4 c0 = mine[0], c1 = mine[1], c2 = mine[2], c3 = mine[3];
        acc += c0.x + c0.y + c0.z + c0.w + c1.x + c1.y + c1.z + c1.w + c2.x + c2.y + c2.z + c3.x + c3.y + c3.z;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the reads are done before the next round overwrites
        r = (r + 1031u) & m;
    }
    sink[blockIdx.x * 64u + lane] = acc;
}

int main() {
    const uint32_t table_f4 = (2u << 20) / 16u, iters = 4096, blocks = 256 * 20 * 4;
    std::vector<float> host(size_t(table_f4) * 4);
    for (size_t i = 0; i < host.size(); ++i) host[i] = float((i * 2654435761u) >> 20) * 1e-3f;
    float4* table = nullptr;
    float* sink = nullptr;
    if (hipMalloc(&table, size_t(table_f4) * 16) != hipSuccess || hipMalloc(&sink, size_t(blocks) * 64 * 4) != hipSuccess)
        return 1;
    (void)hipMemcpy(table, host.data(), size_t(table_f4) * 16, hipMemcpyHostToDevice);
    std::vector<float> s0(size_t(blocks) * 64), s1(s0.size());
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (uint32_t group : {1u, 2u, 4u, 8u, 64u}) {
        float ms_k[3];
        std::vector<float> s2(s0.size());
        for (int k = 0; k < 3; ++k) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(a);
                if (k == 0)
                    hipLaunchKernelGGL(records<false>, dim3(blocks), dim3(64), 0, 0, table, iters, table_f4, sink, group);
                else if (k == 1)
                    hipLaunchKernelGGL(records<true>, dim3(blocks), dim3(64), 0, 0, table, iters, table_f4, sink, group);
                else
                    hipLaunchKernelGGL(records_lds, dim3(blocks), dim3(64), 0, 0, table, iters, table_f4, sink, group);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            ms_k[k] = best;
            (void)hipMemcpy(k == 0 ? s0.data() : k == 1 ? s1.data() : s2.data(), sink, s0.size() * 4,
                            hipMemcpyDeviceToHost);
        }
        const bool same = s0 == s1 && s0 == s2;
        const double steps = double(blocks) * iters * 64;
        printf("{\"lanes_per_record\": %u, \"per_lane_ms\": %.3f, \"quad_ms\": %.3f, \"per_lane_steps_per_ns\": %.1f, "
               "\"quad_steps_per_ns\": %.1f, \"lds_ms\": %.3f, \"lds_steps_per_ns\": %.1f, \"same_sums\": %s}\n",
               group, ms_k[0], ms_k[1], steps / (ms_k[0] * 1e6), steps / (ms_k[1] * 1e6), ms_k[2],
               steps / (ms_k[2] * 1e6), same ? "true" : "false");
    }
    (void)hipFree(table);
    (void)hipFree(sink);
    return 0;
}
