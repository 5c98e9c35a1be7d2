// Internal declarations shared by ggs_kernels.hip and ggs_capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ggs.h"

namespace ggs {

// One preprocessed splat as the raster kernel consumes it (64 B, HBM + LDS).
// cx, cy: centre in pixels (render.py:15-16); A, Bc, Cc, la: exp2-domain
// coefficients of the Gaussian (render.py:189-192 folded with log2(a));
// r, g, b: colour in [0,1] (render.py:40-42); x0..y1: inclusive integer AABB
// (render.py:27-30).
struct __attribute__((aligned(16))) SplatRec {
    float cx, cy, A, Bc;
    float Cc, la, r, g;
    float b, pad0, pad1, pad2;
    int x0, x1, y0, y1;
};
static_assert(sizeof(SplatRec) == 64, "SplatRec must be 64 bytes");

hipError_t launch_prep(hipStream_t st, bool encode, const float* genomes, int64_t S, int C, int H,
                       int W, float k, SplatRec* recs, float* f9, int* i4, float* enc9);
int raster_tiles(int H, int W, int* nTX);
hipError_t launch_raster(hipStream_t st, int mode, const SplatRec* recs, int B, int N, int H, int W,
                         const float bg[3], float* img, const float* target, const float* mask,
                         float beta, float* partials, float* wpartials, const int* tile_order);
// Tile visiting order for the raster grid: tiles sorted by distance of their
// centre from the image centre (central tiles carry the most splats; running
// them first shortens the tail of the launch).
void raster_tile_order(int H, int W, int* order);
hipError_t launch_detmath(hipStream_t st, const float* x, const float* y, int64_t n, int fn,
                          float* out);
hipError_t launch_finalize(hipStream_t st, const float* partials, const float* wpartials, int B,
                           int nTiles, int mode, int H, int W, float* out);

}  // namespace ggs
