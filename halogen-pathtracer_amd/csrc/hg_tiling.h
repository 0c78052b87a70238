// hg_tiling.h — the image tiling of the multi-GPU path, one definition for device and host code.
//
// The image is cut into 8x8 tiles numbered row-major (g = ty * tiles_x + tx).  Rank r of n owns the tiles g with
// g % n == r, stored in its accumulator as local tile l = g / n (tile-major, pixel (x & 7) + 8 (y & 7) of a tile at
// float4 l * 64 + lane; hg_layout.h).  The gather moves every rank's local tiles into slab r of the root's staging
// buffer ([rank][slab_tiles][64] float4, slab_tiles = rank 0's count, the largest).  hg_assemble_image (hg_comm.hip)
// and its host twin hg_comm_assemble_host (the torch-gather path of halogen/distributed.py and the CPU tests) both
// read the image through hg_pixel_source, so the two gathers cannot disagree on where a pixel lives.
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define HG_HD __host__ __device__ __forceinline__
#else
#define HG_HD inline
#endif

// tiles owned by `rank` of n when the image has `total` tiles (ragged: the first total % n ranks hold one more)
HG_HD int64_t hg_rank_tiles(int64_t total, int32_t rank, int32_t n) {
    return total > rank ? (total - rank + n - 1) / n : 0;
}

struct HgPixelSource {
    uint32_t rank;        // owner rank of the pixel's tile
    uint32_t local_tile;  // the tile's index in that rank's accumulator / slab
    uint32_t lane;        // the pixel within the tile, (x & 7) + 8 (y & 7)
};

// Where image pixel (x, y) lives among the ranks' tiles
HG_HD HgPixelSource hg_pixel_source(uint32_t x, uint32_t y, uint32_t tiles_x, uint32_t n_ranks) {
    const uint32_t g = (y >> 3) * tiles_x + (x >> 3);
    return HgPixelSource{g % n_ranks, g / n_ranks, (x & 7u) + 8u * (y & 7u)};
}

// float4 index of a pixel source in the [rank][slab_tiles][64] staging layout
HG_HD size_t hg_slab_index(const HgPixelSource& s, uint32_t slab_tiles) {
    return (size_t(s.rank) * slab_tiles + s.local_tile) * 64u + s.lane;
}
