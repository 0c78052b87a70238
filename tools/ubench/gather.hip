// Micro-benchmark: random 64-B record gathers, per-lane (4 x dwordx4 per lane) vs quad-cooperative
// (each lane of a 4-lane group loads one 16-B chunk of a record; 4 instructions fetch the 4 quad-mates'
// records; then a 4x4 transpose through DPP gives every lane its own 64-B record).  Same records, same math.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <chrono>

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

// naive: each lane chases its own pointer chain, loads its whole 64-B record itself
__global__ void naive(const float4* __restrict__ rec, uint32_t n, int steps, float* out) {
    uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t idx = hash(tid) % n;
    float acc = 0.f;
    for (int s = 0; s < steps; ++s) {
        const float4* r = rec + 4 * idx;
        float4 a = r[0], b = r[1], c = r[2], d = r[3];
        acc += a.x + b.y + c.z + d.w;
        idx = (__float_as_uint(a.w) ^ __float_as_uint(d.x)) % n;  // dependent next index
    }
    out[tid] = acc;
}

__device__ __forceinline__ float quad_get(float v, int src) {  // value of lane (quad base + src)
    return __shfl(v, (threadIdx.x & ~3) + src, 64);
}

// cooperative: lane (4g+p) loads chunk p of quad-mate i's record in step i
__global__ void coop(const float4* __restrict__ rec, uint32_t n, int steps, float* out) {
    uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int p = threadIdx.x & 3;
    uint32_t idx = hash(tid) % n;
    float acc = 0.f;
    for (int s = 0; s < steps; ++s) {
        float4 c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t mate = __shfl(idx, (threadIdx.x & ~3) + i, 64);
            c[i] = rec[4 * mate + p];  // chunk p of mate i's record
        }
        // lane p holds chunk p of all 4 mates' records; my record's chunk q lives in lane q, slot c[p]
        float4 mine[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            // from lane q take c[my p]: lane q must provide c[p_target]; use per-lane select of source slot
            float4 v;
            // each lane sends c[j] where j = requester's position: do 4 rounds of shuffles
            v.x = __shfl(c[0].x, 0, 64); // placeholder, replaced below
            mine[q] = v;
        }
        // correct transpose: round r: every lane sends c[(p + r) & 3] to lane base + ((p + r) & 3)...
        float4 res[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int send_slot = (p + r) & 3;          // I hold chunk p of mate send_slot's record
            float4 sv = c[0];
            if (send_slot == 1) sv = c[1];
            if (send_slot == 2) sv = c[2];
            if (send_slot == 3) sv = c[3];
            // lane (base + send_slot) receives it: it gets chunk ((its p - r) & 3)
            const int src = (threadIdx.x & ~3) + ((p - r) & 3);
            float4 rv;
            rv.x = __shfl(sv.x, src, 64); rv.y = __shfl(sv.y, src, 64);
            rv.z = __shfl(sv.z, src, 64); rv.w = __shfl(sv.w, src, 64);
            const int chunk = (p - r) & 3;               // chunk index of my own record received this round
            if (chunk == 0) res[0] = rv;
            if (chunk == 1) res[1] = rv;
            if (chunk == 2) res[2] = rv;
            if (chunk == 3) res[3] = rv;
        }
        acc += res[0].x + res[1].y + res[2].z + res[3].w + 0.0f * mine[0].x;
        idx = (__float_as_uint(res[0].w) ^ __float_as_uint(res[3].x)) % n;
    }
    out[tid] = acc;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : (1u << 20);  // records (64 B each)
    const int steps = 32;
    std::vector<float4> h(size_t(n) * 4);
    for (size_t i = 0; i < h.size(); ++i) {
        uint32_t a = uint32_t(i * 2654435761u);
        h[i] = make_float4(1.f, 2.f, 3.f, __builtin_bit_cast(float, a & 0x7fffffff));
    }
    float4* d; float* out;
    hipMalloc(&d, h.size() * 16); hipMemcpy(d, h.data(), h.size() * 16, hipMemcpyHostToDevice);
    const int threads = 256 * 8 * 256;
    hipMalloc(&out, threads * 4);
    for (int variant = 0; variant < 2; ++variant) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            if (variant == 0) hipLaunchKernelGGL(naive, dim3(threads / 256), dim3(256), 0, 0, d, n, steps, out);
            else hipLaunchKernelGGL(coop, dim3(threads / 256), dim3(256), 0, 0, d, n, steps, out);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            double recs = double(threads) * steps;
            printf("%s n=%u: %.3f ms, %.2f G records/s (%.1f GB/s of records)\n", variant ? "coop " : "naive", n, ms,
                   recs / ms / 1e6, recs * 64 / ms / 1e6);
        }
    }
    return 0;
}
