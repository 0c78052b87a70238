// hg_mega.hip — the one-thread-per-pixel megakernel (variant HG_KERNEL_MEGA).
//
// Reference: Assets/Scripts/Halogen Shaders/HalgoenCompute.compute, kernel HalogenCompute (:1015-1063) with
// the accumulation blit (AccumulationShader.shader:27-34) fused as its epilogue.  One wave64 = one 8x8 pixel
// tile, each lane runs all n_frames frames of its pixel back to back, the BLAS stack lives in LDS
// ([depth][lane]).  It is the simplest faithful form of the hot path; the runtime uses it for the debug
// views (modes 1-5 need per-path TriangleTests/AABBTests) and as the A/B baseline of the wavefront pipeline
// (hg_wavefront.hip), which is the default for rendering.
#include <hip/hip_runtime.h>

#include "hg_device.h"

using namespace hgd;

template <bool kCounters>
__global__ __launch_bounds__(256, HG_MEGA_WAVES) void hg_trace_kernel(const HgKernelParams kp) {
    extern __shared__ uint32_t lds_stack[];
    const uint32_t lane = threadIdx.x & 63u;
    const int local_tile = int(blockIdx.x) * int(blockDim.x >> 6) + int(threadIdx.x >> 6);
    const int gtile = kp.rank + local_tile * kp.n_ranks;
    const uint32_t px = uint32_t(gtile % kp.tiles_x) * HG_TILE + (lane & 7u);
    const uint32_t py = uint32_t(gtile / kp.tiles_x) * HG_TILE + (lane >> 3);
    const bool active = local_tile < kp.n_local_tiles && px < kp.Wu && py < kp.Hu;
    Counters c{0, 0, 0, 0, 0, 0};
    uint32_t paths = 0;
    if (active) {
        uint32_t* stack = lds_stack + threadIdx.x;
        const uint32_t stride = blockDim.x;
        const size_t slot = size_t(local_tile) * 64 + lane;
        float4 acc = kp.acc[slot];
        // HalogenCompute :1023-1033
        const float ndcx = (float(px) / kp.W) * 2.0f - 1.0f;
        const float ndcy = (float(py) / kp.H) * 2.0f - 1.0f;
        const uint32_t pixel_id = pcg_hash(px + py * kp.Wu);
        for (int f = 0; f < kp.n_frames; ++f) {
            const int32_t fc = kp.accumulate ? kp.first_frame + f : 1;
            Sampler smp{uint32_t(fc), pixel_id, 0u};
            MediumStack ms{0ull, 0};
            f3 color = mk(0, 0, 0);
            for (uint32_t s = 0; s < kp.spp; ++s) {
                const Ray r = camera_ray(kp, smp, ndcx, ndcy);
                paths++;
                if (kp.debug_mode < 1) color = color + trace_ray(kp, smp, ms, r, c, stack, stride);
                else color = color + trace_ray_debug(kp, smp, ms, r, c, stack, stride);
            }
            const float sppf = float(kp.spp);
            color = mk(color.x / sppf, color.y / sppf, color.z / sppf);
            if (kp.accumulate) {  // AccumulationShader.shader:33, w = 1/FrameCount
                const float w = 1.0f / float(fc);
                const float k = 1.0f - w;
                acc.x = acc.x * k + color.x * w;
                acc.y = acc.y * k + color.y * w;
                acc.z = acc.z * k + color.z * w;
                acc.w = acc.w * k + 1.0f * w;
            } else {
                acc = make_float4(color.x, color.y, color.z, 1.0f);
            }
        }
        kp.acc[slot] = acc;
    }
    if (kCounters) {
        const uint32_t v[7] = {paths, c.rays, c.tri, c.aabb, c.meshes, c.spheres, c.hits};
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const uint32_t s = wave_sum(v[k]);
            if (lane == 0 && s) atomicAdd(kp.counters + k, (unsigned long long)s);
        }
    }
}

// Launcher used by the runtime (hg_runtime.hip)
hipError_t hg_launch_mega(const HgKernelParams& kp, int block, bool counters, hipStream_t stream) {
    const int tiles_per_block = block / 64;
    const int grid = (kp.n_local_tiles + tiles_per_block - 1) / tiles_per_block;
    if (grid == 0) return hipSuccess;
    const size_t lds = size_t(kp.stack_depth) * size_t(block) * sizeof(uint32_t);
    if (counters)
        hipLaunchKernelGGL(hg_trace_kernel<true>, dim3(grid), dim3(block), lds, stream, kp);
    else
        hipLaunchKernelGGL(hg_trace_kernel<false>, dim3(grid), dim3(block), lds, stream, kp);
    return hipGetLastError();
}
