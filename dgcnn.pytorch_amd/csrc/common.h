// Shared helpers for the dgx HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dgx.h"

#define DGX_WAVE 64

#define DGX_CHECK_LAUNCH()                                  \
    do {                                                    \
        if (hipGetLastError() != hipSuccess) return DGX_ELAUNCH; \
    } while (0)

static inline hipStream_t dgx_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// XCD-aware block -> work-item map (MI355X_MICROARCH.md: blocks b and b+8 share
// an XCD). Items are (cloud, tile) pairs; all tiles of one cloud get the same
// block residue mod 8 so the cloud's rows are served from one XCD's L2:
// grid = 8 * ceil(B/8) * tiles. A batch of fewer than 8 clouds (a strong-scaling
// shard) would leave 8 - B XCDs with padding blocks only, so there each cloud
// takes rep = 8 / B XCDs, each a contiguous range of ceil(tiles / rep) of its
// tiles: grid = 8 * ceil(tiles / rep). Returns false for padding blocks.
__host__ __device__ __forceinline__ int dgx_xcd_rep(int B) { return B >= 8 ? 1 : 8 / B; }
__device__ __forceinline__ bool dgx_xcd_cloud_map(int block, int B, int tiles, int& b, int& tile) {
    const int xcd = block & 7, r = block >> 3;
    const int rep = dgx_xcd_rep(B);
    if (rep == 1) {
        const int bl = r / tiles;
        tile = r - bl * tiles;
        b = bl * 8 + xcd;
        return b < B;
    }
    const int per = (tiles + rep - 1) / rep;
    b = xcd / rep;
    tile = (xcd - b * rep) * per + r;
    return b < B && r < per && tile < tiles;
}
static inline int dgx_xcd_cloud_grid(int B, int tiles) {
    const int rep = dgx_xcd_rep(B);
    return rep == 1 ? 8 * ((B + 7) / 8) * tiles : 8 * ((tiles + rep - 1) / rep);
}

// (cloud, point part, channel slice) work items of the EdgeConv gather/scatter
// kernels: every block of one cloud gets the same residue mod 8 (one XCD) and
// consecutive dispatch slots, so the slices that read different 32-64 B pieces
// of the same rows run together and the rows come from HBM once (that XCD's
// L2 serves the rest). Slices vary fastest. Returns false for padding blocks.
__device__ __forceinline__ bool dgx_xcd_slice_map(int block, int B, int parts, int slices, int& b, int& part,
                                                  int& slice) {
    int tile;
    if (!dgx_xcd_cloud_map(block, B, parts * slices, b, tile)) return false;
    part = tile / slices;
    slice = tile - part * slices;
    return true;
}

// LeakyReLU shared by the EdgeConv (edgeconv.hip) and edge-MLP (edgemlp.hip) kernels.
__device__ __forceinline__ float lrelu(float v, float slope) { return v > 0.f ? v : v * slope; }
