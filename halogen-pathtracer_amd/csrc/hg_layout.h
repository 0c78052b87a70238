// hg_layout.h — device-side data layout of the Halogen scene in HBM (private to libhalogen_hip.so).
//
// The ABI structs (include/halogen_abi.h) are the reference's AoS C# layouts.  hg_upload_scene repacks
// them once into the layout below, chosen for the gfx950 traversal loop:
//
//   node records   64 B per BLAS entry, CHILD-PAIR form: record g holds the boxes of g's two children and
//                  their node refs, so popping an inner node costs exactly one 64-B record fetch (4 x
//                  dwordx4) and the reference's re-read of the popped node (HalgoenCompute.compute:405)
//                  disappears.  Records of leaf entries are never read.
//   leaf table     8 B per BLAS entry: (global first triangle, triangle count) — read only for leaves.
//   node ref       uint32: bit 31 = leaf, bits 0..30 = global BLAS index (= accelerationBufferOffset +
//                  mesh-relative index).  Decided at upload from triangleCount, so the kernel never has to
//                  read a node to know what it is.
//   triangles      36 B per triangle, packed (v0.xyz, e1.xyz, e2.xyz), where e1 = v1 - v0 and e2 = v2 - v0 are the
//                  reference's own first two subtractions (:312-313) done once on the host with the same IEEE
//                  operation; a leaf's triangles sit on 2-3 cache lines.
//   normals        48 B per triangle (n0, n1 - n0, n2 - n0), read once per accepted hit.
//   meshes         144 B per mesh (HgDevMesh): full worldToLocal (16 floats, Unity column-major), root ref,
//                  triangle offset, material index, the exact-cull boxes.
//   spheres        48 B: (centre, radius), (cornerA, material bits), (cornerB, 0).
//   materials      80 B: albedo; (specular.rgb, metallic); (emissive.rgb*intensity, roughness);
//                  (absorption.xyz, ior); (priority, medium id, roughness^2, 0).
//   accumulation   float4 per pixel, TILE-MAJOR: 8x8 tiles of 1 KiB, local tile t holds global tile
//                  rank + t*n_ranks, pixel (lx,ly) at lx + 8*ly — one wave writes one contiguous KiB.
//
// The measured-and-rejected experiments of rounds 1-4 (wavefront pipeline, path pool, LDS node cache, quad /
// deduplicated node fetch, ray sort, path migration, packed-pair and stream triangle layouts, ...) were removed from
// the sources in round 5; their designs and numbers stay in DESIGN.md section 10 and in git history.
#pragma once
#include <stdint.h>

#define HG_LEAF_BIT 0x80000000u
// Leaf refs: HG_LEAF_BIT | count << HG_LEAF_CNT_SHIFT | first triangle, for leaves of 1..15 triangles starting
// below 2^27 (no memory access to find a leaf's range); count field 0: the low bits index the leaf table instead.
#define HG_LEAF_CNT_SHIFT 27
#define HG_LEAF_INLINE_MAX 15u
#define HG_LEAF_PAYLOAD ((1u << HG_LEAF_CNT_SHIFT) - 1u)
#define HG_TILE 8
#define HG_MAX_CUBE_MIPS 16
#define HG_REGEN_MAX_BOUNCES 250  // regenerating megakernel: byte-packed bounce counters (larger: lockstep kernel)
#define HG_REGEN_MAX_CHUNK 65535  // regenerating megakernel: frames per launch and spp limit (16-bit fields)
#ifndef HG_LOCK_WAVES
#define HG_LOCK_WAVES 4  // lockstep megakernel (debug views, large-maxBounces fallback): waves/SIMD target
#endif
#ifndef HG_MEGA_WAVES
#define HG_MEGA_WAVES 6  // regenerating megakernel: waves/SIMD target
#endif
#ifndef HG_STREAM_WAVES
#define HG_STREAM_WAVES 5  // streaming kernel: waves/SIMD target (its resumable traversal state needs ~96 VGPRs)
#endif
#ifndef HG_STREAM_TMIN
#define HG_STREAM_TMIN 16  // streaming kernel: shade once at most this many lanes are still traversing (12 before the
                           // item scheduling, tools/sweeps/sweep54.txt; 16 with it, +1.1 %, tools/sweep_r02_ac.txt)
#endif
#ifndef HG_DESCENT_T
#define HG_DESCENT_T 3  // deep scenes (BLAS depth > HG_DESCENT_DEEP): leave the descent loop at <= T descending lanes
#endif
#ifndef HG_STREAM_TMIN_DEEP
#define HG_STREAM_TMIN_DEEP 20  // ... for a deep BLAS (C3 +0.6 %, C3F +1.0 %, strict 1-frame +1.5 %; C2 keeps 16: -1.2 %;
#endif                          // tools/sweeps/sweep_r04_results.txt)
#ifndef HG_STREAM_RESHADE_DEEP
#define HG_STREAM_RESHADE_DEEP 24
#endif
#ifndef HG_STREAM_RESHADE
#define HG_STREAM_RESHADE 16  // streaming kernel: repeat the shading pass while at least this many lanes need it
#endif
#ifndef HG_STREAM_DESCENT_T
#define HG_STREAM_DESCENT_T 12  // the same for the streaming kernel (tools/sweeps/sweep42.txt; 8 with the unsplit launch,
                                // sweep74; 12 with the in-place item scheduling, +2.4 %, tools/sweep_r02_al.txt)
#endif
#ifndef HG_DESCENT_DEEP
#define HG_DESCENT_DEEP 16
#endif
// Wave priorities (s_setprio): the streaming kernel's waves run at 1 while traversing (traversal waits on memory: its
// waves issue first) and 0 while shading (C3 2,097 -> 2,111, tools/sweeps/sweep67-68.txt); the regenerating kernel's
// at 1 during get_ray_intersection (C2 +1 %, C5 +2 %, tools/sweeps/sweep69.txt).
#define HG_TRAVERSE_PRIO 1
#ifndef HG_TILE_ORDER
#define HG_TILE_ORDER 1  // regen / stream kernels: dispatch tiles in descending cost of the previous launch (hg_order_tiles)
#endif
#ifndef HG_ORDER_MIN_FRAMES
#define HG_ORDER_MIN_FRAMES 16  // hg_render re-sorts the tile order once at least this many frames of costs were recorded
#endif                          // since the last sort (64-frame launches: every launch; 1-frame launches: every 16th)
// Every mesh's world->local matrix and header (80 B) in the wave's LDS when they fit (mesh_lds_bytes): the per-lane
// mesh switch reads LDS, not global memory
#define HG_MESH_LDS_F4 5  // float4 per cached mesh record: w2l columns 0-3, header (root, tri offset, material, cull)
// Bytes of LDS per one-wave workgroup that still keep 20 waves (5 per SIMD) on a CU.  Measured, not derived from
// 160 KiB / 20: 7,424 and 7,472 B run at full occupancy, 7,936 / 7,984 / 8,192 B lose 8-12 % (one wave fewer per
// CU; tools/sweep_r02_h.txt); 7,680 is the largest multiple of 512 below the first failing size.
#ifndef HG_WAVE_LDS_BUDGET
#define HG_WAVE_LDS_BUDGET 7680
#endif
#ifndef HG_REGEN_LDS_BUDGET
// The same for the regenerating kernel at its 6 waves per SIMD (24 per CU): 163,840 / 24 = 6,826, less the same
// reserve; 0 keeps its mesh records in global memory
#define HG_REGEN_LDS_BUDGET 6144
#endif
#ifndef HG_COALESCE
#define HG_COALESCE 32  // default HG_OPT_COALESCE: frames of consecutive hg_render calls held for one launch
#endif
#ifndef HG_TRACE_LANES
#define HG_TRACE_LANES 12  // trace streams of the render pipeline (hg_ctx.h): chunks traced in turn on them, blended in
#endif                    // order.  1-frame launches, C3, all waves per launch: 2 streams 1,970, 3: 2,143, 4: 2,265,
                          // 6: 2,242, 8: 2,302 Mpaths/s; with HG_QUEUE_WAVES_DIV 6 and 8 streams 2,745, with 8 and 10 / 12
                          // streams 2,808 / 2,790 (tools/sweeps/sweep_r03_u/v/y/z/aa; streams 3+ on hardware queues of
                          // their own).  Round 4 (queue heads reset in-kernel, small sort), streams / divisor 8/6
                          // 2,779-2,793, 12/8 2,874-2,878, 12/12 2,748-2,753, 16/12 2,893-2,908, 16/16 2,800-2,808
                          // (tools/sweeps/sweep_r04_a.txt): 12/8, +3 % for four more queues per context
#ifndef HG_TRACE_LANES_BIG
#define HG_TRACE_LANES_BIG 2  // of those, the ones chunks of more than HG_QUEUE_MAX_FRAMES frames take in turn (a third
#endif                        // 64-frame launch beside two others: C3 -1.5 %)
// Trace streams: HIP spreads plain streams over a pool of GPU_MAX_HW_QUEUES (default 4) hardware queues shared by every
// stream of the process, and two streams on one queue run their launches one after the other (a third plain trace
// stream cost 1-frame launches 16 %: 1,663 vs 1,970).  A stream created with a CU mask gets a hardware queue of its
// own: the first HG_TRACE_LANES_BIG trace streams are plain and non-blocking, the others (and the render server's and
// the side copy stream) carry an all-CU mask (create_lane_stream, hg_runtime.hip).
#ifndef HG_QUEUE_WAVES_DIV
#define HG_QUEUE_WAVES_DIV 8  // queue launches beside >= 2 other traces in flight: at most this many times fewer persistent
#endif                        // waves than resident slots (hg_render; C3 1-frame launches, 8 streams: 1 2,265 -> 6 2,745;
                              // 12 streams: 8 2,874-2,878, 12 2,748-2,753)
#ifndef HG_READBACK_SIDE
#define HG_READBACK_SIDE 0  // default HG_OPT_READBACK_STREAM (display copies on a side stream)
#endif
#ifndef HG_WAVE_UNITS_MAX
#define HG_WAVE_UNITS_MAX 1     // streaming launches without the queue: at most this many tiles per wave (automatic)
#endif
#ifndef HG_WAVE_UNITS_ROUNDS
#define HG_WAVE_UNITS_ROUNDS 3  // ... while the launch keeps at least this many waves per resident wave slot
#endif
#ifndef HG_LANE_PICK
#define HG_LANE_PICK 1  // default HG_OPT_LANE_PICK (display one frame behind +5 %, strict -0.5 %: sweep_r04_depth)
#endif
#define HG_WAVE_UNITS_LIMIT 4  // HG_OPT_WAVE_UNITS range (the units' tiles sit in scalar registers)
#ifndef HG_QUEUE_FILL
// default HG_OPT_QUEUE_FILL: streaming launches of more than HG_QUEUE_MAX_FRAMES frames whose tiles give fewer rounds of
// the GPU's wave slots than this run the queue form (a rank's share at N = 8, 1080p: 0.79 rounds).  With about 24
// (tile, frame chunk) units per wave slot the queue form costs 6 % against per-tile waves at N = 1 (C3: 3,288 vs 3,491
// Mpaths/s); emulated shares, queue vs per-tile: N = 2 3,229 vs 3,366, N = 4 3,114 vs 3,122, N = 8 2,937 vs 2,803
#define HG_QUEUE_FILL 1
#endif
#define HG_QUEUE_FILL_UNITS 24  // queue-form shares: (tile, frame chunk) units per wave slot
#ifndef HG_SHARE_HOLD_ROUNDS
// A rank's share of the image (hg_set_tiling, N > 1) holds consecutive hg_render calls (HG_OPT_COALESCE > 1) until the
// held launch has this many rounds of the GPU's wave slots in 64-frame tile waves, as one context's 64-frame launch of
// the whole 1080p image has (32,400 tiles / 5,120 slots): 8 calls of 64 frames at N = 8, 4 at N = 4, 2 at N = 2.
// Emulated strong shares of C3 (tools/gpu_strong_coalesce.sh): N = 8 3,000 -> 3,526 Mpaths/s, N = 4 3,128 -> 3,465.
#define HG_SHARE_HOLD_ROUNDS 6
#endif
#define HG_SHARE_HOLD_MAX 1024  // frames: the most a share holds (its frame colours: 2 trace streams x 4 GiB at most)
#ifndef HG_QUEUE_MAX_FRAMES
#define HG_QUEUE_MAX_FRAMES 8  // streaming launches of at most this many frames run the persistent work-queue form (kQueue)
#endif
// The queue of a kQueue launch: 8 unit heads, 128 B apart (words 32 h), then the count of waves that have left (its own
// 128-B line): the last wave out zeroes them for the next launch (the runtime zeroes the buffer once, at allocation)
#define HG_QUEUE_DONE_WORD 256u
#define HG_QUEUE_BYTES (9u * 128u)
// Render server control words (kp.queue of a server launch, HG_SV_CTL_BYTES, zeroed at each server start), each on a
// 128-B line of its own: the 8 unit heads (as above), then HG_SV_MIRRORS copies of the device mirror of the host's post
// word (u64, raised by atomic max by whichever wave read the host word; an idle
// wave reads copy blockIdx.x % HG_SV_MIRRORS: the polling of thousands of idle waves spread over as many lines), one
// host-poll ticket per XCD (blockIdx.x % 8), the count of waves that left (read by the gates: a frame whose count is
// short once every wave has left is lost), and the closing word (0 open, 1 closing: the one wave that won it runs the
// close handshake, hg_mega.hip sv_close)
#define HG_SV_MIRRORS 16u
#define HG_SV_MIRROR_WORD 288u
#define HG_SV_TICKET_WORD (HG_SV_MIRROR_WORD + 32u * HG_SV_MIRRORS)
#define HG_SV_EXIT_WORD (HG_SV_TICKET_WORD + 32u * 8u)  // waves of the server that left | grid << 32
#define HG_SV_CLOSE_WORD (HG_SV_EXIT_WORD + 32u)
#ifndef HG_SV_DIAG_TIMES
#define HG_SV_DIAG_TIMES 0  // analysis builds: per frame (< 256) the device time of its first claim and its last count
#endif
#define HG_SV_DIAG_WORD (HG_SV_CLOSE_WORD + 32u)
#define HG_SV_CTL_BYTES ((HG_SV_DIAG_WORD + (HG_SV_DIAG_TIMES ? 1024u : 0u)) * 4u)
#ifndef HG_SV_POLL_TICKS
#define HG_SV_POLL_TICKS 200u  // 2 us between reads of the host word over PCIe, per XCD
#endif
#ifndef HG_SV_SLEEP_LONG  // an idle server wave's wait between polls: HG_SV_SPIN_SHORT spins of s_sleep SHORT, then LONG
#define HG_SV_SLEEP_SHORT 8
#define HG_SV_SLEEP_LONG 127
#define HG_SV_SPIN_SHORT 16u
#define HG_SV_POLL_EVERY 4u  // an idle wave reads the host word (if its XCD's ticket is free) every this many spins
#endif
#ifndef HG_SV_WAVES
#define HG_SV_WAVES 5  // the render server's persistent waves per SIMD (hg_runtime.hip server_start)
#endif
#ifndef HG_SV_COST_ORDER
// The render server's units in the cost order of its last lifetime's frames (1) or in raster order with no cost records
// (0).  The cost order puts a launch's longest tiles first so that its end waits less on them; the server's frames
// overlap, so there is no such end, and raster order keeps a claim's consecutive tiles together.  C3, server forced,
// one box, two rounds (tools/sweeps/sweep_r06_server_order.txt): strict 3,155 / 3,159 -> 3,168 / 3,164, display at once (R11G11B10F)
// 2,662 / 2,669 -> 2,752 / 2,726 Mpaths/s.
#define HG_SV_COST_ORDER 0
#endif
#ifndef HG_SV_TILE_RUN
// The render server's XCD heads take runs of this many consecutive tiles (hg_mega.hip sv_pull): head h (the XCD whose
// waves pull it first) runs h, h + 8, ..., so a CU's waves pull neighbouring tiles and the heads still interleave
// finely over the frame (one contiguous band per head lost 1-3 %: per-XCD balance).  C3, server forced, one box, two
// rounds (tools/sweeps/sweep_r06_server_runs.txt), runs of 1 / 4 / 8 / 16: strict 3,169-3,176 / 3,183-3,194 /
// 3,187-3,193 / 3,181-3,183, display at once 2,643-2,714 / 2,706-2,716 / 2,724-2,735 / 2,701, one behind
// 2,811-2,847 / 2,837-2,868 / 2,879-2,881 / 2,789-2,862 Mpaths/s.
#define HG_SV_TILE_RUN 8u
#endif
#ifndef HG_SV_CLAIM
#define HG_SV_CLAIM 4u  // units per claim of a server wave far behind the posted units (the rest held for its next pulls)
#endif
#ifndef HG_SV_RING
#define HG_SV_RING 16  // colour ring slots of the render server (frames traced ahead of their blend), at most
#endif
#define HG_SV_STOP (1ull << 32)  // the post word's stop flag (posted frames in the low 32 bits)
// The host words of a server (pinned, coherent; u64 each): the post word (frames posted | HG_SV_STOP), the lost-frame
// word (a gate that gave up: HG_SV_LOST | the accumulator epoch of its frame), the closing word (raised by the wave
// that closes the server, before it reads the post word) and the close word (the post word as that wave read it, with
// HG_SV_STOP, | HG_SV_CLOSED once written)
#define HG_SV_HOST_POST 0
#define HG_SV_HOST_LOST 1
#define HG_SV_HOST_CLOSING 2
#define HG_SV_HOST_CLOSED 3
#define HG_SV_CLOSED (1ull << 33)
#define HG_SV_LOST (1ull << 32)
#ifndef HG_SV_AHEAD
#define HG_SV_AHEAD 4  // default HG_OPT_SERVER_AHEAD: frames the render server traces ahead of the host's calls (4 and 8 measured equal)
#endif
#define HG_SV_IDLE_US 200000  // default HG_OPT_SERVER_IDLE_US: the server closes after this long with nothing posted
#ifndef HG_REGEN_ITEMS
#define HG_REGEN_ITEMS 1  // regenerating kernel: (pixel, frame) item scheduling (0: the A/B build of make noitems)
#endif
#ifndef HG_STREAM_MIN_MESHES
#define HG_STREAM_MIN_MESHES 4  // HG_KERNEL_AUTO: the streaming kernel from this many meshes on (or for a deep BLAS)
#endif
#ifndef HG_STREAM_LB
#define HG_STREAM_LB 64  // regen / stream kernels: __launch_bounds__ max threads = their one-wave workgroup (256: scratch 32 B vs 24-28 B)
#endif
#ifndef HG_CHECK_EXEC
#define HG_CHECK_EXEC 0  // debug builds: leaf_dist checks its all-lanes-active precondition (hg_device.h)
#endif
#ifndef HG_MEGA_LDS_STACK
#define HG_MEGA_LDS_STACK 16  // megakernels: traversal stack entries per lane kept in LDS (deeper ones spill)
#endif
#ifndef HG_STREAM_LDS_STACK
#define HG_STREAM_LDS_STACK 12  // the same for the streaming kernel (12 and 14 measured equal, 10 equal to 16 without the
                                // mesh records in LDS; 12 leaves LDS room for 16 meshes, HG_WAVE_LDS_BUDGET)
#endif

struct alignas(16) HgDevMesh {
    float w2l[16];  // Unity column-major: column c = w2l[4c .. 4c+3]
    uint32_t root_ref;
    uint32_t tri_offset;
    uint32_t material;
    uint32_t cullable;  // 1: the root is an inner node and cull_* hold its children's padded world boxes
    // World-space boxes of the root's two children, padded far beyond every float rounding of the reference's
    // local-space test (hg_runtime.hip: mesh_cull_boxes).  If a ray certainly misses both (or meets them only
    // beyond its current closest hit), the reference's traversal of this mesh would test exactly those two
    // boxes, push nothing and find nothing — so the mesh is skipped and only its 2 AABB tests are counted.
    float4 cull_a_lo, cull_a_hi, cull_b_lo, cull_b_hi;
};

// Everything the trace kernel needs, passed by value as the kernel argument.
struct HgKernelParams {
    // camera (rows 0..2 of CamLocalToWorldMatrix, row-major: cam[r*4+c] = M(r,c))
    float cam[12];
    float W, H;
    uint32_t Wu, Hu;
    float vw, vh, near_, far_;
    float focal_disc_radius;  // tan(radians(focalConeAngle)) * near, evaluated on the host with hg_fmath.h
    float psx, psy;           // (vw*2)/W, (vh*2)/H
    float filter_radius, focal_dist;
    uint32_t spp, max_bounces, max_diff, max_glossy, max_trans;
    uint32_t debug_mode, tri_range, box_range;
    int32_t default_mip;
    int32_t use_cube;
    int32_t n_spheres, n_meshes;
    int32_t first_frame, n_frames, accumulate;
    // frame-parallel split (regenerating kernel): frame_split waves share each tile, wave k tracing frames
    // [k*n_frames/split, (k+1)*n_frames/split) into frame_color (fc_index); hg_blend_frames then applies the
    // accumulation blend in frame order.  frame_split == 1: the kernel blends into acc itself.
    int32_t frame_split;
    float4* __restrict__ frame_color;  // render server: a ring of sv_ring frames, frame k at [(k & (sv_ring-1)) * slots]
    // render server (kServer): per ring slot a completion count on its own 128-B line (word 32 s), advanced by
    // n_local_tiles for every frame of that slot; the context stream's gate waits for it (hg_server_gate)
    uint32_t* __restrict__ frames_done;
    // cost-ordered dispatch (regen / stream kernels): wave w traces local tile tile_order[w % n_local_tiles] (null:
    // tile w % n_local_tiles) and adds its wave-clock cost to tile_cost[tile] (null: not recorded).  Any permutation
    // gives the same image: tiles are independent and each tile's frames keep their order.
    unsigned long long* __restrict__ tile_cost;  // s_memtime cycles per tile
    const uint32_t* __restrict__ tile_order;
    // HG_STREAM_QUEUE: 8 unit heads (one per XCD, 128 B apart: queue[32 h]), zeroed before each streaming launch, and
    // the number of persistent waves (one per resident wave slot of the GPU)
    uint32_t* __restrict__ queue;
    uint32_t resident_waves;
    // streaming launches without the queue and without a frame split: each wave traces wave_units consecutive units
    // of the cost order (1: one tile per wave), its lanes taking their items one after another (UnitItems)
    uint32_t wave_units;
    // render server: the host words in pinned host memory (HG_SV_HOST_*; [0] the post word, frames posted | stop << 32)
    const unsigned long long* __restrict__ sv_post;
    uint32_t sv_ring;        // colour ring slots (a power of two)
    uint32_t sv_frames_cap;  // frames the server may trace in its lifetime (n_local_tiles * frames < 2^31)
    uint32_t sv_idle_ticks;  // nothing posted for this long (100-MHz s_memrealtime ticks): a wave closes the server
    uint32_t sv_div_magic, sv_div_shift;  // unit -> frame: u / n_local_tiles = umulhi(u, magic) >> shift (u < 2^31)
    // tiling
    int32_t tiles_x, rank, n_ranks, n_local_tiles;
    uint32_t stack_depth;  // LDS traversal stack entries per lane
    uint32_t mesh_lds_word;  // the mesh records' LDS copy starts at this word (mesh_lds_bytes, hg_mega.hip)
    uint32_t descent_t;    // relaxed while-while threshold (hg_device.h isect_meshes), 0 = classic while-while
    uint32_t stream_deep;  // streaming kernel: the deep-BLAS shading thresholds (HG_STREAM_TMIN_DEEP / _RESHADE_DEEP)
    uint32_t* __restrict__ spill;  // per-lane traversal stack entries beyond the LDS part (rarely touched)
    uint32_t spill_stride;          // = threads of the launch grid
    // cubemap
    int32_t cube_size, cube_mips;
    uint32_t cube_mip_offset[HG_MAX_CUBE_MIPS];  // in float4 texels
    // scene
    const float4* __restrict__ spheres;
    const HgDevMesh* __restrict__ meshes;
    const float4* __restrict__ materials;
    const float4* __restrict__ nodes;
    const uint2* __restrict__ leaves;
    const float* __restrict__ tris;  // 9 floats per triangle: v0, e1, e2
    const float4* __restrict__ normals;
    const float4* __restrict__ cube;
    // outputs
    float4* __restrict__ acc;
    unsigned long long* __restrict__ counters;  // 32 x u64: 0-6 hg_counters' first 7 fields, 7-15 wave-level
                                                // rounds / clocks, 16 primary misses (hg_runtime.hip hg_get_counters)
};

#define HG_NONE 0xFFFFFFFFu
#define HG_SPHERE_BIT 0x80000000u
