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

// kDebug: the debug views (HalogenDebugMode 1-5) get their own instantiation so the production kernel's register
// allocation does not pay for trace_ray_debug.
template <bool kCounters, bool kDebug>
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
                if (!kDebug) color = color + trace_ray(kp, smp, ms, r, c, stack, stride);
                else color = color + trace_ray_debug(kp, smp, ms, r, c, stack, stride);
            }
            const float sppf = float(kp.spp);
            color = mk(color.x / sppf, color.y / sppf, color.z / sppf);
            float4 acc = kp.acc[slot];  // read-modify-write per frame: 32 B, keeps 4 VGPRs free while tracing
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
            kp.acc[slot] = acc;
        }
    }
    if (kCounters) {
        // every ray transforms into every mesh and prefilters every sphere: those counts follow from c.rays
        const uint32_t v[7] = {paths, c.rays, c.tri, c.aabb, c.rays * uint32_t(kp.n_meshes),
                               c.rays * uint32_t(kp.n_spheres), c.hits};
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const uint32_t s = wave_sum(v[k]);
            if (lane == 0 && s) atomicAdd(kp.counters + k, (unsigned long long)s);
        }
    }
}

// Regenerating variant (HG_KERNEL_MEGA_REGEN): each loop iteration runs ONE bounce (get_ray_intersection + one
// body of trace_ray's loop) for every lane; a lane whose path ended starts its next sample / frame right away
// (blending the finished frame into the accumulator), so lanes never wait for the longest path of their wave —
// at the price of desynchronising the lanes' bounce depths (less coherent node fetches).
template <bool kCounters>
__global__ __launch_bounds__(256, HG_MEGA_WAVES) void hg_trace_regen_kernel(const HgKernelParams kp) {
    extern __shared__ uint32_t lds_stack[];
    const uint32_t lane = threadIdx.x & 63u;
    const int local_tile = int(blockIdx.x) * int(blockDim.x >> 6) + int(threadIdx.x >> 6);
    const int gtile = kp.rank + local_tile * kp.n_ranks;
    const uint32_t px = uint32_t(gtile % kp.tiles_x) * HG_TILE + (lane & 7u);
    const uint32_t py = uint32_t(gtile / kp.tiles_x) * HG_TILE + (lane >> 3);
    bool work = local_tile < kp.n_local_tiles && px < kp.Wu && py < kp.Hu && kp.n_frames > 0;
    Counters c{0, 0, 0, 0, 0, 0};
    uint32_t paths = 0;
    uint32_t* stack = lds_stack + threadIdx.x;
    const uint32_t stride = blockDim.x;
    const size_t slot = size_t(local_tile) * 64 + lane;
    const float ndcx = (float(px) / kp.W) * 2.0f - 1.0f;
    const float ndcy = (float(py) / kp.H) * 2.0f - 1.0f;
    const uint32_t pixel_id = pcg_hash(px + py * kp.Wu);
    uint32_t f = 0, s = 0, iter = 0;
    Sampler smp{uint32_t(kp.accumulate ? kp.first_frame : 1), pixel_id, 0u};
    MediumStack ms{0ull, 0};
    Ray ray{mk(0, 0, 0), mk(0, 0, 1)};
    f3 thr = mk(1, 1, 1), col = mk(0, 0, 0), sum = mk(0, 0, 0);
    float acc_rough = 0.0f;
    Bounces bounce{0, 0, 0};
    if (work) {
        ray = camera_ray(kp, smp, ndcx, ndcy);
        paths++;
    }
    while (__any(work)) {
        if (work) {
            const Hit hit = intersect(kp, ray, c, stack, stride);
            bool alive = false;
            if (hit.t < kp.far_) {  // :898-936
                c.hits++;
                const Mat mt = load_mat(kp, hit.mat);
                col = col + xyz(mt.emis_rough) * thr;
                const f3 att = evaluate_hit(kp, smp, ms, ray, hit, mt, bounce);
                thr = thr * att;
                acc_rough += mt.emis_rough.w * thr.x;
                const float rr = smp.get1(ID_RR);
                smp.offset += BOUNCE_INC;
                const float contribution = fmaxf(fmaxf(thr.x, thr.y), thr.z);
                if (!(rr > contribution)) {
                    thr = thr * (1.0f / contribution);
                    iter++;
                    alive = iter <= kp.max_bounces && !(bounce.diffuse > kp.max_diff ||
                                                       bounce.glossy > kp.max_glossy ||
                                                       bounce.transmission > kp.max_trans);
                }
            } else {  // :941
                col = col + sample_sky(kp, ray.d, sky_level(kp, acc_rough)) * thr;
            }
            if (!alive) {
                sum = sum + col;  // RayColor += trace_ray(...)
                ++s;
                bool next = s < kp.spp;  // next sample: statics persist (:188-189)
                if (!next) {
                    const float sppf = float(kp.spp);
                    const f3 color = mk(sum.x / sppf, sum.y / sppf, sum.z / sppf);
                    float4 acc = kp.acc[slot];
                    if (kp.accumulate) {
                        const float w = 1.0f / float(smp.frame);
                        const float k = 1.0f - w;
                        acc = make_float4(acc.x * k + color.x * w, acc.y * k + color.y * w, acc.z * k + color.z * w,
                                          acc.w * k + 1.0f * w);
                    } else {
                        acc = make_float4(color.x, color.y, color.z, 1.0f);
                    }
                    kp.acc[slot] = acc;
                    ++f;
                    if (f < uint32_t(kp.n_frames)) {  // next frame = next dispatch: statics reset
                        next = true;
                        s = 0;
                        sum = mk(0, 0, 0);
                        smp.frame = kp.accumulate ? uint32_t(kp.first_frame) + f : 1u;
                        smp.offset = 0;
                        ms = MediumStack{0ull, 0};
                    }
                }
                if (next) {
                    ray = camera_ray(kp, smp, ndcx, ndcy);
                    thr = mk(1, 1, 1);
                    col = mk(0, 0, 0);
                    acc_rough = 0.0f;
                    bounce = Bounces{0, 0, 0};
                    iter = 0;
                    paths++;
                } else {
                    work = false;
                }
            }
        }
    }
    if (kCounters) {
        const uint32_t v[7] = {paths, c.rays, c.tri, c.aabb, c.rays * uint32_t(kp.n_meshes),
                               c.rays * uint32_t(kp.n_spheres), c.hits};
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const uint32_t sv = wave_sum(v[k]);
            if (lane == 0 && sv) atomicAdd(kp.counters + k, (unsigned long long)sv);
        }
    }
}

hipError_t hg_launch_mega_regen(const HgKernelParams& kp, int block, bool counters, hipStream_t stream) {
    const int tiles_per_block = block / 64;
    const int grid = (kp.n_local_tiles + tiles_per_block - 1) / tiles_per_block;
    if (grid == 0) return hipSuccess;
    const size_t lds = size_t(kp.stack_depth) * size_t(block) * sizeof(uint32_t);
    if (counters)
        hipLaunchKernelGGL(hg_trace_regen_kernel<true>, dim3(grid), dim3(block), lds, stream, kp);
    else
        hipLaunchKernelGGL(hg_trace_regen_kernel<false>, dim3(grid), dim3(block), lds, stream, kp);
    return hipGetLastError();
}

// Launcher used by the runtime (hg_runtime.hip)
hipError_t hg_launch_mega(const HgKernelParams& kp, int block, bool counters, hipStream_t stream) {
    const int tiles_per_block = block / 64;
    const int grid = (kp.n_local_tiles + tiles_per_block - 1) / tiles_per_block;
    if (grid == 0) return hipSuccess;
    const size_t lds = size_t(kp.stack_depth) * size_t(block) * sizeof(uint32_t);
    const bool dbg = kp.debug_mode != 0;
    if (counters && dbg)
        hipLaunchKernelGGL((hg_trace_kernel<true, true>), dim3(grid), dim3(block), lds, stream, kp);
    else if (counters)
        hipLaunchKernelGGL((hg_trace_kernel<true, false>), dim3(grid), dim3(block), lds, stream, kp);
    else if (dbg)
        hipLaunchKernelGGL((hg_trace_kernel<false, true>), dim3(grid), dim3(block), lds, stream, kp);
    else
        hipLaunchKernelGGL((hg_trace_kernel<false, false>), dim3(grid), dim3(block), lds, stream, kp);
    return hipGetLastError();
}
