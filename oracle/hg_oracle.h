/*
 * hg_oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of the Halogen hot path, used as the parity
 * checker (tests/, __graft_entry__.smoke) and as bench.py's cpu_baseline.  The product path
 * (libhalogen_hip.so) never links, loads or calls anything under oracle/.
 *
 * Parity status: UNPINNED against the reference's own outputs — the reference (HLSL + C# in Unity) has
 * no tests, no golden images and cannot be compiled or run in this image (no dxc/Unity/dotnet).  What is
 * pinned: the Sobol direction table (against the Joe–Kuo construction and against the table text in
 * HalogenRandom.hlsl:10-46, tests/golden/sobol_table.json), the sampler hashes (against an independent
 * numpy restatement), and the transcendental spec (include/hg_fmath.h, against libm to <= 2 ulp).
 */
#ifndef HG_ORACLE_H
#define HG_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#include "halogen_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hgo_scene {
    const HalogenSphere* spheres;
    int32_t n_spheres;
    const HalogenMeshData* meshes;
    int32_t n_meshes;
    const PackedHalogenMaterial* materials;
    int32_t n_materials;
    const HalogenTriangle* triangles;
    int32_t n_triangles;
    const BVHEntry* blas;
    int32_t n_nodes;
    /* cubemap, layout as hg_upload_cubemap; NULL when absent */
    const float* cube_texels;
    int32_t cube_face_size;
    int32_t cube_mips;
} hgo_scene;

/* Sampler (HalogenRandom.hlsl) */
uint32_t hgo_pcg_hash(uint32_t v);
uint32_t hgo_hash_combine(uint32_t seed, uint32_t v);
uint32_t hgo_owen_scramble(uint32_t value, uint32_t seed);
uint32_t hgo_sobol1d(uint32_t index, uint32_t dim);
uint32_t hgo_sobol_table(uint32_t dim, uint32_t bit);
uint32_t hgo_u32_owen_scrambled_sobol(uint32_t index, uint32_t dimension, uint32_t seed);
void hgo_u32_2d_owen_scrambled_sobol(uint32_t index, uint32_t dimension, uint32_t seed, uint32_t out[2]);
float hgo_inverted_blackman_harris(float x);

/* BVHGenerator.GenerateMeshBVH restated (BVHGenerator.cs:13-200) */
int64_t hgo_build_blas(const float* vertices, int32_t n_vertices, int32_t* indices, int32_t n_tris,
                       const float root_min[3], const float root_max[3], int32_t max_depth,
                       BVHEntry* out_nodes, int64_t max_nodes);

/* Render n_frames frames into acc (row-major W*H*4 floats) for pixels [pix_begin, pix_end) in row-major
 * order, FrameCount = params->frameCount + k, blend as AccumulationShader.shader:33.  Counters summed into
 * `counters` (may be NULL).  n_threads >= 1. */
int hgo_render(const hgo_scene* scene, const hg_params* params, int32_t n_frames, int32_t accumulate,
               float* acc, int64_t pix_begin, int64_t pix_end, int32_t n_threads, hg_counters* counters);

/* One path of pixel (x,y) for debugging single-pixel parity: returns RayColor/SPP in rgb[3]. */
void hgo_trace_pixel(const hgo_scene* scene, const hg_params* params, uint32_t x, uint32_t y, int32_t frame,
                     float rgb[3], hg_counters* counters);

/* Diagnostics, collected only by the stats build (HGO_STATS=1: build/libhgoracle_stats.so; the plain build keeps
 * the traversal free of them and reports zeros, max_depth -1).  hgo_stats_build() says which build this is.
 * Mesh traversals (since the last reset) whose node stack would hold more than the reference's NodeStack[32]
 * entries (HC:397), and the deepest stack seen. */
int hgo_stats_build(void);
void hgo_stack_stats(uint64_t* overflow_traversals, int32_t* max_depth, int32_t reset);
/* Diagnostics: inner-node visits by the number of children the exact test keeps: [root 0/1/2, inner 0/1/2]. */
void hgo_visit_stats(uint64_t out[6], int32_t reset);

/* Per-stage KAT entry points */
float hgo_sphere_t(const float o[3], const float d[3], const float c[3], float r);
float hgo_triangle_t(const float o[3], const float d[3], const float v0[3], const float v1[3], const float v2[3],
                     float* u, float* v, float* orientation);
float hgo_aabb_t(const float a[3], const float b[3], const float o[3], const float inv_d[3]);
void hgo_cube_sample(const hgo_scene* scene, const float dir[3], int32_t level, float rgb[3]);
/* Seamless cube filtering: the adjacent face's texel for texel (i, j) one step outside face f (out: face, i, j). */
void hgo_cube_adjacent(int32_t f, int32_t i, int32_t j, int32_t size, int32_t out[3]);
void hgo_fmath(int32_t fn, const float* x, float* y, int64_t n);

#ifdef __cplusplus
}
#endif
#endif
