/* TEST INFRASTRUCTURE: a standalone driver of the CPU oracle for sanitizer builds (make -C oracle sanitize:
 * AddressSanitizer + UndefinedBehaviorSanitizer, every report fatal).  tests/test_sanitizers.py runs it.
 *
 *   hg_oracle_asan render SCENE.hgscene PARAMS.bin FRAMES THREADS OUT.f32 [CUBE.hgcube]
 *       the reference-layout scene (halogen/host_files.py write_scene), the raw hg_params block, FRAMES progressive
 *       frames on THREADS pthreads; writes the RGBA32F image (compared bit for bit with the unsanitized oracle)
 *   hg_oracle_asan blas N_TRIS SEED
 *       hgo_build_blas (BVHGenerator.cs restated) on a random soup of N_TRIS triangles, every triangle in one leaf
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hg_oracle.h"

static void* read_file(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", path); exit(2); }
    fseek(f, 0, SEEK_END);
    long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    void* buf = malloc((size_t)len);
    if (!buf || fread(buf, 1, (size_t)len, f) != (size_t)len) { fprintf(stderr, "read %s failed\n", path); exit(2); }
    fclose(f);
    *n = (size_t)len;
    return buf;
}

static int render(int argc, char** argv) {
    if (argc < 7) return 2;
    size_t n_scene, n_params;
    uint8_t* scene = read_file(argv[2], &n_scene);
    hg_params* params = read_file(argv[3], &n_params);
    if (n_params != sizeof(hg_params) || n_scene < 28 || memcmp(scene, "HGSCENE1", 8) != 0) return 3;
    const int32_t* cnt = (const int32_t*)(scene + 8);
    const size_t sizes[5] = {sizeof(HalogenSphere), sizeof(HalogenMeshData), sizeof(PackedHalogenMaterial),
                             sizeof(HalogenTriangle), sizeof(BVHEntry)};
    /* copy every array into its own exact-size allocation, so an overrun of any of them is caught */
    void* arr[5];
    size_t off = 28;
    for (int k = 0; k < 5; k++) {
        const size_t bytes = (size_t)cnt[k] * sizes[k];
        if (off + bytes > n_scene) return 3;
        arr[k] = malloc(bytes ? bytes : 1);
        memcpy(arr[k], scene + off, bytes);
        off += bytes;
    }
    hgo_scene sc;
    memset(&sc, 0, sizeof sc);
    sc.spheres = arr[0];
    sc.n_spheres = cnt[0];
    sc.meshes = arr[1];
    sc.n_meshes = cnt[1];
    sc.materials = arr[2];
    sc.n_materials = cnt[2];
    sc.triangles = arr[3];
    sc.n_triangles = cnt[3];
    sc.blas = arr[4];
    sc.n_nodes = cnt[4];
    float* cube = NULL;
    if (argc > 7) {
        size_t n_cube;
        uint8_t* c = read_file(argv[7], &n_cube);
        if (memcmp(c, "HGCUBE01", 8) != 0) return 3;
        int32_t face, mips;
        int64_t n_floats;
        memcpy(&face, c + 8, 4);
        memcpy(&mips, c + 12, 4);
        memcpy(&n_floats, c + 16, 8);
        cube = malloc((size_t)n_floats * sizeof(float));
        memcpy(cube, c + 24, (size_t)n_floats * sizeof(float));
        sc.cube_texels = cube;
        sc.cube_face_size = face;
        sc.cube_mips = mips;
        free(c);
    }
    const int frames = atoi(argv[4]), threads = atoi(argv[5]);
    const int64_t W = (int64_t)params->screenParameters.x, H = (int64_t)params->screenParameters.y;
    float* acc = calloc((size_t)(W * H * 4), sizeof(float));
    hg_counters counters;
    memset(&counters, 0, sizeof counters);
    if (hgo_render(&sc, params, frames, 1, acc, 0, W * H, threads, &counters) != 0) return 4;
    FILE* out = fopen(argv[6], "wb");
    if (!out || fwrite(acc, sizeof(float), (size_t)(W * H * 4), out) != (size_t)(W * H * 4)) return 5;
    fclose(out);
    printf("rendered %lldx%lld x%d frames: %llu rays, %llu triangle tests\n", (long long)W, (long long)H, frames,
           (unsigned long long)counters.rays, (unsigned long long)counters.tri_tests);
    for (int k = 0; k < 5; k++) free(arr[k]);
    free(cube);
    free(acc);
    free(scene);
    free(params);
    return 0;
}

static uint32_t rng_state;
static float rnd(void) { /* xorshift32 in [0, 1) */
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 17;
    rng_state ^= rng_state << 5;
    return (float)(rng_state >> 8) / 16777216.0f;
}

static int blas(int argc, char** argv) {
    if (argc < 4) return 2;
    const int32_t n_tris = atoi(argv[2]);
    rng_state = (uint32_t)atoi(argv[3]) | 1u;
    const int32_t n_verts = 3 * n_tris;
    float* v = malloc((size_t)n_verts * 3 * sizeof(float));
    int32_t* idx = malloc((size_t)n_tris * 3 * sizeof(int32_t));
    float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
    for (int32_t t = 0; t < n_tris; t++) {
        const float cx = rnd() * 10.0f, cy = rnd() * 10.0f, cz = rnd() * 10.0f;
        for (int k = 0; k < 3; k++) {
            float* p = v + (3 * t + k) * 3;
            p[0] = cx + rnd() * 0.2f;
            p[1] = cy + rnd() * 0.2f;
            p[2] = cz + rnd() * 0.2f;
            for (int a = 0; a < 3; a++) {
                if (p[a] < lo[a]) lo[a] = p[a];
                if (p[a] > hi[a]) hi[a] = p[a];
            }
            idx[3 * t + k] = 3 * t + k;
        }
    }
    const int64_t cap = 2 * (int64_t)n_tris + 1;
    BVHEntry* nodes = malloc((size_t)cap * sizeof(BVHEntry));
    const int64_t n = hgo_build_blas(v, n_verts, idx, n_tris, lo, hi, 32, nodes, cap);
    if (n <= 0) return 6;
    int32_t* seen = calloc((size_t)n_tris, sizeof(int32_t));
    for (int64_t i = 0; i < n; i++)
        for (uint32_t k = 0; k < nodes[i].triangleCount; k++) seen[nodes[i].indexA + k]++;
    for (int32_t t = 0; t < n_tris; t++)
        if (seen[t] != 1) { fprintf(stderr, "triangle %d in %d leaves\n", t, seen[t]); return 7; }
    printf("built %lld BVH entries over %d triangles\n", (long long)n, n_tris);
    free(seen);
    free(nodes);
    free(idx);
    free(v);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && strcmp(argv[1], "render") == 0) return render(argc, argv);
    if (argc > 1 && strcmp(argv[1], "blas") == 0) return blas(argc, argv);
    fprintf(stderr, "usage: %s render SCENE PARAMS FRAMES THREADS OUT [CUBE] | blas N_TRIS SEED\n", argv[0]);
    return 2;
}
