// Per-splat prep math shared by the prep kernel (ggs_kernels.hip) and the GA's
// variation kernel (ggs_ga.hip, which preps the offspring it writes):
//   encode_row      encode.py:4-59   axes-angle row -> renderer row
//   preprocess_row  render.py:8-47   renderer row -> centre, inverse covariance,
//                                    colours, integer AABB
//   make_rec        raster coefficients (exp2 domain) + row-recurrence constants
//   finalize_wave   fitness.py:17-31 normalisation of one candidate's strip sums
// Bounds-critical math uses ggs_detmath.h (bit-exact with oracle/detmath.py);
// every TU including this is compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>

#include "ggs_detmath.h"
#include "ggs_internal.h"

namespace ggs {

using namespace detmath;

struct Prep13 {
    float cx, cy, sxx, sxy, syy, rc, gc, bc, a;
    int x0, x1, y0, y1;
};

// encode.py:4-24 + 27-59: axes-angle row -> renderer row (g2, g3, g4 replaced,
// colours/alpha clamped).  Same op order as oracle/ggs_oracle.py.
__device__ __forceinline__ void encode_row(const float* __restrict__ g, float out[9]) {
    const float sx = det_expf(g[2]);
    const float sy = det_expf(g[3]);
    float s, c;
    det_sincosf(g[4], &s, &c);
    const float sx2 = sx * sx, sy2 = sy * sy, c2 = c * c, s2 = s * s;
    const float sxx = sx2 * c2 + sy2 * s2;
    const float sxy = ((sx2 - sy2) * s) * c;
    const float syy = sx2 * s2 + sy2 * c2;
    const float l11 = ggs_sqrt_rn(nmax(sxx, EPS12));
    const float l21 = ggs_div_rn(sxy, l11);
    const float l22 = ggs_sqrt_rn(nmax(syy - l21 * l21, EPS12));
    out[0] = g[0];
    out[1] = g[1];
    out[2] = det_logf(l11);
    out[3] = det_logf(l22);
    out[4] = l21;
#pragma unroll
    for (int j = 5; j < 9; ++j) out[j] = nclamp(g[j], 0.0f, 255.0f);
}

// render.py:8-47 on one renderer row.
__device__ __forceinline__ Prep13 preprocess_row(const float g[9], int H, int W, float k) {
    Prep13 p;
    const float maxx = (float)(W - 1), maxy = (float)(H - 1);
    p.cx = nclamp(g[0], 0.0f, 1.0f) * maxx;
    p.cy = nclamp(g[1], 0.0f, 1.0f) * maxy;
    const float l11 = nmax(det_expf(g[2]), EPS6);
    const float l22 = nmax(det_expf(g[3]), EPS6);
    const float l21 = g[4];
    const float hx = nmax(k * fabsf(l11), 1.0f);
    const float hy = nmax(k * (fabsf(l21) + fabsf(l22)), 1.0f);
    p.x0 = (int)floorf(nclamp(p.cx - hx, 0.0f, maxx));
    p.x1 = (int)ceilf(nclamp(p.cx + hx, 0.0f, maxx));
    p.y0 = (int)floorf(nclamp(p.cy - hy, 0.0f, maxy));
    p.y1 = (int)ceilf(nclamp(p.cy + hy, 0.0f, maxy));
    const float i11 = ggs_div_rn(1.0f, l11);
    const float i22 = ggs_div_rn(1.0f, l22);
    const float i21 = (-l21) * (i11 * i22);
    p.sxx = i11 * i11 + i21 * i21;
    p.sxy = i21 * i22;
    p.syy = i22 * i22;
    p.rc = ggs_div_rn(nclamp(g[5], 0.0f, 255.0f), 255.0f);
    p.gc = ggs_div_rn(nclamp(g[6], 0.0f, 255.0f), 255.0f);
    p.bc = ggs_div_rn(nclamp(g[7], 0.0f, 255.0f), 255.0f);
    p.a = ggs_div_rn(nclamp(g[8], 0.0f, 255.0f), 255.0f);
    return p;
}

// Raster coefficients.  exp(-0.5*quad)*a == exp2(e) with
// e = K*(sxx qx^2 + 2 sxy qx qy + syy qy^2) + log2(a),  K = -0.5*log2(e).
// The cull's copy of a record's AABB: a compact [B][N] int4 array (16 B per
// splat; the 64-B records of 1,024-splat candidates overflowed the XCD L2s when
// every strip-wave's cull walked them, 1024^2 config).
__device__ __forceinline__ int4 rec_bounds(const SplatRec& r) { return make_int4(r.x0, r.x1, r.y0, r.y1); }

__device__ __forceinline__ SplatRec make_rec(const Prep13& p) {
    constexpr float K = -0.72134752044448170f;
    SplatRec r;
    r.cx = p.cx;
    r.A = K * p.sxx;
    const float Bc = 2.0f * K * p.sxy, Cc = K * p.syy;
    // the raster's y-side in qy / 8: e = (qy/8) (64 Cc (qy/8) + 8 Bc qx) + px is
    // e = qy (Cc qy + Bc qx) + px with every operand scaled by a power of two, so
    // every rounding is the same (the same bits), and the row ratio's exponent
    // d = 16 Cc (qy + 4) + 8 Bc qx is one FMA, 128 Cc (qy + 4)/8 + 8 Bc qx
    r.cy8 = 0.125f * p.cy;
    r.B8 = 8.0f * Bc;
    r.C64 = 64.0f * Cc;
    r.la = p.a > 0.0f ? __builtin_amdgcn_logf(p.a) : -__builtin_inff();
    r.r = p.rc;
    r.g = p.gc;
    r.b = p.bc;
    // f(qy + 8) = f(qy) * 2^d(qy),  d(qy) = e(qy + 8) - e(qy) = 16 Cc (qy + 4) + 8 bx,
    // d(qy + 8) = d(qy) + 128 Cc  ->  the raster walks rows with two multiplies;
    // d(qy + 4) = d(qy) + 64 Cc   ->  the pair's second row ratio is one multiply.
    r.rho = __builtin_amdgcn_exp2f(128.0f * Cc);
    r.c128 = 128.0f * Cc;
    r.rho4 = __builtin_amdgcn_exp2f(64.0f * Cc);
    r.x0 = p.x0;
    r.x1 = p.x1;
    r.y0 = p.y0;
    r.y1 = p.y1;
    // The raster seeds its row recurrence with the exact value of a visit's first
    // row pair and walks a thin rotated splat exactly instead when a live seed is
    // below 2^-100.  Seeds lie in columns [x0, x1] and rows [y0 - 7, y1]; e is
    // concave along both axes (A, Cc <= 0), so its minimum over that rectangle is
    // at a corner.  A splat whose corner minimum is at least 2^-99 can never trip
    // the check: the raster skips it (one margin unit covers the rounding
    // difference between this and the raster's FMA form of e).  The flag is the
    // sign bit of rho4 (the raster takes |rho4|): set = run the check.
    float emin = __builtin_inff();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float qx = (float)((c & 1) ? p.x1 : p.x0) - r.cx;
        const float qy = (float)((c & 2) ? p.y1 : p.y0 - 7) - p.cy;
        const float e = qy * (Cc * qy + Bc * qx) + (r.A * qx * qx + r.la);
        emin = fminf(emin, e);
    }
    if (!(emin >= -99.0f)) r.rho4 = -r.rho4;     // NaN too
    return r;
}

// fitness.py:17-31 for one candidate, by one wave: lane l sums x[l], x[l+64], ...
// in order (float64), then a fixed xor butterfly (every lane ends with the same
// bits: a+b == b+a).  Strip partials give the numerator, the plan's per-strip
// weight sums the denominator.  finalize_kernel and the GA's survivors kernel
// both call this, so the fitness of a candidate has the same bits either way.
// COHERENT: the partials were written by waves of the SAME launch, possibly on
// other XCDs (the raster's fused finalize): agent-scope loads (sc1) read them at
// the device coherence point, past this XCD's L2.  Same adds, same bits.
template <bool COHERENT = false>
__device__ __forceinline__ float ld_partial(const float* __restrict__ p) {
    if (COHERENT) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return *p;
}
template <bool COHERENT = false>
__device__ __forceinline__ double wave_sum(const float* __restrict__ x, int n) {
    // lane from mbcnt, not threadIdx.x: the raster's folded finalize would
    // otherwise keep threadIdx.x live (and spilled) across its epilogue
    const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    double a = 0.0;
    int i = lane;
    // loads in flight in blocks (32, then 8), then the same in-order adds: the
    // bits do not depend on the blocking (2,048 strip partials at 2048^2 were 32
    // dependent HBM round trips per lane: 16 us per finalize; 4 with blocks of 8)
    for (; i + 31 * 64 < n; i += 32 * 64) {
        float v[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) v[k] = ld_partial<COHERENT>(x + i + k * 64);
#pragma unroll
        for (int k = 0; k < 32; ++k) a += (double)v[k];
    }
    for (; i + 7 * 64 < n; i += 8 * 64) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = ld_partial<COHERENT>(x + i + k * 64);
#pragma unroll
        for (int k = 0; k < 8; ++k) a += (double)v[k];
    }
    for (; i < n; i += 64) a += (double)ld_partial<COHERENT>(x + i);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
    return a;
}

template <bool COHERENT = false>
__device__ __forceinline__ float finalize_wave(const float* __restrict__ partials,
                                               const float* __restrict__ wpartials, int nT, int mode,
                                               double hw, int b) {
    const double num = wave_sum<COHERENT>(partials + (int64_t)b * nT, nT);
    // wpartials: the plan's weight block, Sum w (float64) first (plan_wsum_kernel)
    const double wsum = mode != GGS_FIT_NONE ? *reinterpret_cast<const double*>(wpartials) : 0.0;
    double v;
    if (mode == GGS_FIT_NONE) v = num / (3.0 * hw);                       // fitness.py:18-19
    else if (mode == GGS_FIT_WEIGHTED) v = num / (wsum + 1e-12);          // fitness.py:28-31
    else v = (num / (3.0 * hw)) / (wsum / hw + 1e-12);                    // fitness.py:23-27
    return (float)v;
}

}  // namespace ggs
