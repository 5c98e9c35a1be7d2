// MI355X (gfx950) kernels for the 2D Gaussian-splat render + fitness hot path.
//
// Replaces, behind the reference's interfaces:
//   encode      genome_to_renderer_batched         modules/encode.py:4-79
//   preprocess  _preprocess_genome                 modules/render.py:8-47
//   binning     _gpu_bin_splats_to_tiles           modules/render.py:50-118
//   raster      _render_tile_over_kernel (Triton)  modules/render.py:121-200
//   epilogue    canvas fill / clamp / L2 fitness   modules/render.py:235-252, fitness.py:16-31
//
// Three launches per batch (fitness) — prep, raster, finalize; two for render;
// plus plan once per fitness target.
//   prep     1 thread / splat: encode (fitness) + preprocess -> 64-B SplatRec in HBM.
//            Bounds-critical math is ggs_detmath.h (bit-exact with oracle/).
//   raster   1 wave64 / (candidate, 64x128 tile, 16-column strip).  Order-preserving
//            cull of the candidate's N splats against the strip (wave ballot +
//            mbcnt compaction, no global sort) into an LDS list, then a front-to-
//            back per-pixel blend: lane (c, r) owns column c and rows r, r+4, ...,
//            r+124 (32 pixels held in registers, two rows per packed op).  Per
//            splat the x-dependent half of the Gaussian exponent is formed once
//            per lane; the first row pair gets the exact exponent, further pairs
//            a multiplicative row recurrence (no exp); row ranges outside the
//            splat's AABB are skipped wave-uniformly.  Epilogue: background +
//            clamp, then either the image store (render) or the weighted squared
//            error against the target plan, summed per strip (the image never
//            touches HBM).
//   finalize fixed-order float64 sum of a candidate's strip partials -> the
//            fitness scalar (deterministic: the order never depends on which
//            wave finished last).  Folded into the raster where the caller
//            hands it a counter block (FinFused: the candidate's last strip
//            wave reduces), else its own launch, one wave per candidate.
//   plan     1 wave / (tile, strip): target + mode weights in raster lane order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <utility>
#include <vector>

#include "ggs_detmath.h"
#include "ggs_internal.h"
#include "ggs_prep.h"

// The raster's folded finalize (strip_done) relies on gfx9-family store/vmcnt
// semantics and the wave64 layout; this file is written for gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "ggs_kernels.hip targets gfx950 (MI355X) only"
#endif

namespace ggs {

using namespace detmath;

// ---------------------------------------------------------------------------
// prep (per-splat math in ggs_prep.h, shared with the GA's fused variation)
// ---------------------------------------------------------------------------
template <bool ENCODE>
__global__ void __launch_bounds__(256)
prep_kernel(const float* __restrict__ genomes, int64_t S, int C, int H, int W, float k,
            SplatRec* __restrict__ recs, int4* __restrict__ bnds, float* __restrict__ f9, int* __restrict__ i4,
            float* __restrict__ enc9, const int* __restrict__ live, int n_per) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S) return;
    if (live && i >= (int64_t)*live * n_per) return;   // SA loop: candidates past the round's count
    const float* g = genomes + i * (int64_t)C;
    float row[9];
    if (ENCODE) {
        encode_row(g, row);
    } else {
#pragma unroll
        for (int j = 0; j < 9; ++j) row[j] = g[j];
    }
    if (enc9) {
#pragma unroll
        for (int j = 0; j < 9; ++j) enc9[i * 9 + j] = row[j];
    }
    const Prep13 p = preprocess_row(row, H, W, k);
    if (recs) {
        const SplatRec r = make_rec(p);
        recs[i] = r;
        bnds[i] = rec_bounds(r);
    }
    if (f9) {
        f9[0 * S + i] = p.cx;  f9[1 * S + i] = p.cy;  f9[2 * S + i] = p.sxx;
        f9[3 * S + i] = p.sxy; f9[4 * S + i] = p.syy; f9[5 * S + i] = p.rc;
        f9[6 * S + i] = p.gc;  f9[7 * S + i] = p.bc;  f9[8 * S + i] = p.a;
    }
    if (i4) {
        i4[0 * S + i] = p.x0; i4[1 * S + i] = p.x1; i4[2 * S + i] = p.y0; i4[3 * S + i] = p.y1;
    }
}

// ---------------------------------------------------------------------------
// raster
// ---------------------------------------------------------------------------
constexpr int TILE = 64;          // tile width (pixels): 4 strips of 16 columns
#ifndef GGS_TILE_H
#define GGS_TILE_H 128            // probe build only: other strip heights (multiples of 8)
#endif
constexpr int TILE_H = GGS_TILE_H;  // tile height: one wave covers a 16 x 128 strip, 32 pixels per lane
                                  // (round 1: 64 rows at 5 waves/SIMD 0.260 ms, 96 at 4: 0.249, 128 at 3: 0.249)
constexpr int RG = TILE_H / 4;    // row groups per lane (rows r, r+4, ...)
constexpr int NPK = RG / 2;       // packed row-group pairs per lane
constexpr int WPB = 1;            // one wave per workgroup, one 16-column strip each (2 or 4 waves:
                                  // +1.4 %, +2.5 % raster time, round 1)
constexpr int NT = 64 * WPB;      // threads per workgroup
constexpr int SPB = 4 / WPB;      // workgroups per (candidate, tile)
constexpr int CAP = 1024;         // LDS list capacity per wave (splats per cull round)
constexpr int OCC = 3;            // waves per SIMD the register budget is sized for (<= 168 VGPRs)
// candidate rotation across the XCDs advances every 2^XCD_SHIFT strip groups (see the grid order)
// (launches with N > SAT_MIN_SPLATS, the raster_kernel<M, true, F> instances; the others
// rotate every group: at 512^2/256 splats the whole launch's records (2.1 MB) and the
// 4-MiB target plan share each XCD's L2, and rotating every group lets each XCD read
// each strip's plan slice once: 54 vs 80 MB of fabric traffic per launch, raster
// -0.5 %; at 1024^2/1024 (33 MB of records) the 8-group rotation is 0.6 % faster)
constexpr int XCD_SHIFT = 3;
constexpr int CULL_PRIO = 2;      // s_setprio while culling (1 and 3 measured the same)

// Depth-split experiment (probe build only, docs/EXPERIMENTS.md §15): the fitness
// instances without the saturation check (N <= SAT_MIN_SPLATS) run two waves per
// strip; wave 0 culls the front half of the splat indices, wave 1 the back half,
// each blends half of the joint list, and wave 0 composes the halves with the
// associative "over" (C = C_f + T_f C_b, T = T_f T_b) through LDS.
#ifndef GGS_DEPTH_SPLIT
#define GGS_DEPTH_SPLIT 0
#endif

#ifndef GGS_NOPLAN
#define GGS_NOPLAN 0      // probe build only (docs/EXPERIMENTS.md §4 traffic split): the epilogue reads no plan
#endif

// Saturation cut-off.  Front to back, a strip's pixels receive Σ_rest T·f·c +
// T_end·bg ≤ T from all the splats still to come (Σ w + T_end = T, c, bg ≤ 1).
// Once every pixel of the strip has T < 2^-24 (half an ulp of 1.0) the wave stops:
// no output can move by more than 2^-24, far inside the 1e-4 bar.  Checked every
// SAT_EVERY visits from the SAT_FIRST-th on (deep lists: 2048²/4096-splat SA
// states, ~400 splats per pixel; a 512²/256 strip list is ~45 long and is not
// checked at all; launches with N <= SAT_MIN_SPLATS run the kernel instance
// without the check).  GGS_SATURATE=0 compiles it out.
#ifndef GGS_SATURATE
#define GGS_SATURATE 1
#endif
constexpr float SAT_EPS = 5.9604645e-8f;   // 2^-24
#ifndef GGS_SAT_EVERY
#define GGS_SAT_EVERY 16
#endif
constexpr int SAT_FIRST = 64, SAT_EVERY = GGS_SAT_EVERY;
constexpr int SAT_MIN_SPLATS = 512;          // launches with fewer splats use the kernel without the check
// With the check on, the cull hands over at most SAT_BATCH listed splats at a time
// (not CAP): a 2048²/4096 strip lists ~500, so the blend of the first batch can meet
// saturation before the cull has scanned the rest of the candidate's splats, and
// the cut skips that part of the cull too.  Each batch re-exposes the first record
// fetch, so small batches lose (tools/probe/sat_batch_ab.sh, raster vs CAP: 2048²
// with 16 candidates 128: +7.2 %, 192: +4.3 %, 256: -4.8 %, 384: -3.0 %; with 2:
// +8.7, +8.6, +1.3, -3.3 %; 1024²/1024: +0.8, +1.2, 0.0, +0.1 %; SA loop at
// configs[4], start of a run, 3 alternated runs: 595 it/s -> 601 with 384, 573 with 256).
#ifndef GGS_SAT_BATCH
#define GGS_SAT_BATCH 384
#endif
#ifndef GGS_SAT_AHEAD
#define GGS_SAT_AHEAD 2
#endif
constexpr int SAT_BATCH = GGS_SAT_BATCH;

__device__ __forceinline__ int ufirst(int v) { return __builtin_amdgcn_readfirstlane(v); }

// A cull-list word of the instances without the saturation check (N <= 512) and
// without the folded finalize: the visit's scalar control, formed by the cull (one
// lane per splat, VALU) instead of per visit (SALU) — the record byte offset i * 64 (bits 6-25) with, in its
// free bits, kB (0-4: the strip's last row pair the AABB reaches, NPK when it
// reaches past the tile), "starts at or above the tile" (5), kA (26-29: the first
// row pair) and "the AABB cuts the strip's 16 columns" (31).  The same integer
// tests on the same bounds, so the same paths: 7 fewer SALU per visit, raster
// -0.5 % at 512^2/256, -0.25 % at the shipped GA launch; the saturation instances
// (2048^2 SA: +1.5 %, the longer cull pays the words) keep plain byte offsets
// (docs/EXPERIMENTS.md §16).
constexpr unsigned VW_ABOVE = 32u, VW_KA = 26, VW_CLIP = 31, VW_OFFSET = 0x03FFFFC0u;
__device__ __forceinline__ int visit_word(int i, const int4& bb, int ty0, int sx0) {
    constexpr int NP = GGS_TILE_H / 8;
    const int dy0 = bb.z - ty0, dy1 = bb.w - ty0;
    const unsigned kA = (unsigned)max(dy0, 0) >> 3;
    const unsigned kB = dy1 >= GGS_TILE_H - 1 ? (unsigned)NP : (unsigned)dy1 >> 3;
    const unsigned above = dy0 <= 0 ? VW_ABOVE : 0u;
    const unsigned clip = max(bb.x - sx0, sx0 + 15 - bb.y) > 0 ? (1u << VW_CLIP) : 0u;
    return (int)(((unsigned)i << 6) | kB | above | (kA << VW_KA) | clip);
}

// One strip's partial (lane 0).  With the fused finalize: an agent-scope store,
// written through to the device coherence point, where the candidate's last wave
// (on any XCD) reads it.  Otherwise a plain store (the finalize launch reads it
// after the kernel boundary): the write-through store of every wave measured
// 16 MB of extra write traffic per 512^2 launch (PMC WRITE_SIZE, 0.45 MB plain).
__device__ __forceinline__ void store_partial(float* p, float v, bool fused) {
    if (fused) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
// The fused finalize (FinFused), after lane 0 stored this strip's partial.  The
// partial is the only data another wave reads, and its agent-scope store is
// written through: waiting for that store (vmcnt(0)) before the count orders it,
// so the add itself is relaxed.  (A release add also writes back the whole L2
// (buffer_wbl2) in every wave: raster 0.159 -> 0.351 ms at 512^2/256/pop 128.)
// The wave whose add completes the candidate's count reduces all its partials
// with agent-scope loads (the same finalize_wave arithmetic as finalize_kernel,
// so the same bits whichever wave is last) and re-arms the counter.
__device__ __forceinline__ void strip_done(const FinFused& fin, const float* partials, int b, int nslots,
                                           int lane) {
    int old = 0;
    if (lane == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        old = __hip_atomic_fetch_add(fin.ctr + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (ufirst(old) != nslots - 1) return;
    // acquire at agent scope in the one wave that reduces: pairs with the other
    // waves' drained write-through stores + count, so the partial loads below
    // cannot be satisfied from before the count (HIP memory model, not only the
    // ISA's vmcnt ordering); one wave per candidate pays it
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const float v = finalize_wave<true>(partials, fin.wpartials, nslots, fin.mode, fin.hw, b);
    if (lane == 0) {
        fin.out[b] = v;
        __hip_atomic_store(fin.ctr + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

#ifndef GGS_TIMING
#define GGS_TIMING 0              // diagnostic build: per-wave phase clocks (tools/probe/wave_timing.py)
#endif
#if GGS_TIMING
constexpr int GGS_TIMING_WAVES = 1 << 16;
// per wave (blockIdx, WPB = 1): realtime start, realtime end (100 MHz), cull,
// visit and epilogue shader clocks, HW_ID | XCC_ID << 24, listed visits, blended visits
__device__ unsigned long long g_ggs_timing[8 * GGS_TIMING_WAVES];
#define GGS_TMARK(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define GGS_TMARK(v)
#endif

// Row limits as wave lane masks.  Lane l owns row phase ph = l >> 4: the rows of
// pair k are 8k + ph (x) and 8k + 4 + ph (y).  Each mask is one per-lane compare
// writing an SGPR pair, applied by one v_cndmask (round 3: -0.6 % raster vs
// building the same masks from shifts and selects on the SALU).
struct PairLanes { uint64_t x, y; };          // rows 8k+ph (x) and 8k+4+ph (y)
// j = y0 - (ty0 + 8k) <= 7: keep lanes whose row >= y0 (ph >= j, ph + 4 >= j)
__device__ __forceinline__ PairLanes rows_from_ph(int j, int ph) {
    return {(uint64_t)__ballot(ph >= j), (uint64_t)__ballot(ph + 4 >= j)};
}
// m = y1 - (ty0 + 8k) >= 0: keep lanes whose row <= y1 (ph <= m, ph + 4 <= m)
__device__ __forceinline__ PairLanes rows_upto_ph(int m, int ph) {
    return {(uint64_t)__ballot(ph <= m), (uint64_t)__ballot(ph + 4 <= m)};
}
#define rows_from(j) rows_from_ph((j), ph)
#define rows_upto(m) rows_upto_ph((m), ph)
__device__ __forceinline__ float keep_if(uint64_t lanes, float f) {
    return __builtin_amdgcn_inverse_ballot_w64(lanes) ? f : 0.0f;
}


// Two adjacent row groups (2k, 2k+1) per lane live in one float2, so qy, the
// quadratic and the blend run as v_pk_{add,fma,mul}_f32 (2 FP32 ops per lane per
// issue); the exp stays per element.  e = K*quad + log2(a) (see make_rec),
// f = 2^e, front-to-back "over":
//   C += T*f*c ; T *= (1 - f)       (== render.py:194-196 run back-to-front)
#define GGS_EXP2(x) __builtin_amdgcn_exp2f(x)
static_assert(NPK <= 16, "walk macros cover 16 pairs");
typedef float f2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2_t fma2(f2_t a, f2_t b, f2_t c) { return __builtin_elementwise_fma(a, b, c); }
#define GGS_PK(k, MASKED)                                                            \
    do {                                                                             \
        const f2_t qy_ = (k) == 0 ? qyv : qyv + (f2_t)(float)(k);  /* no +0 add */    \
        f2_t e_ = GGS_E1(qy_);                                                       \
        if (MASKED) {                                                                \
            if ((unsigned)(8 * (k) - rlo) > rspan) e_.x = -__builtin_inff();         \
            if ((unsigned)(8 * (k) + 4 - rlo) > rspan) e_.y = -__builtin_inff();     \
        }                                                                            \
        f2_t f_;                                                                     \
        f_.x = GGS_EXP2(e_.x);                                                       \
        f_.y = GGS_EXP2(e_.y);                                                       \
        const f2_t w_ = P_T##k * f_;                                                 \
        P_R##k = fma2((f2_t)s.r, w_, P_R##k);                                        \
        P_G##k = fma2((f2_t)s.g, w_, P_G##k);                                        \
        P_B##k = fma2((f2_t)s.b, w_, P_B##k);                                        \
        P_T##k = P_T##k - w_;                                                        \
    } while (0)
// Blend one packed pair with given (row-masked) Gaussian values f.
#define GGS_BLEND(k, F)                                                              \
    do {                                                                             \
        const f2_t w_ = P_T##k * (F);                                                \
        P_R##k = fma2((f2_t)s.r, w_, P_R##k);                                        \
        P_G##k = fma2((f2_t)s.g, w_, P_G##k);                                        \
        P_B##k = fma2((f2_t)s.b, w_, P_B##k);                                        \
        P_T##k = P_T##k - w_;                                                        \
    } while (0)
#define GGS_BLEND_REC(k)                                                             \
    if ((k) < NPK) {                                                                 \
        F2 = F2 * R2;                                                                \
        R2 = R2 * (f2_t)s.rho;                                                       \
        GGS_BLEND(k, F2);                                                            \
    }
// The first pair's ratio to the next: 2^d, d(qy) = 16 Cc (qy + 4) + 8 bx, in the
// record's scaled terms fma((qy + 4)/8, 128 Cc, 8 bx) (the .y row's qy/8).  Live
// lanes of well-formed splats have d <= -e(seed) <= 100 (make_rec's seed guard:
// e <= 0 everywhere), so the clamp is exact there; lanes with f = 0 (outside the
// AABB's columns, or a degenerate splat's: infinite conic terms) only need a
// finite ratio (0 * r = 0), which the clamp gives without a per-lane select
// (round 3: raster -1.0 %, bit-identical).  (Round 4 measured the clamp's
// removal with 8 bx = -1e30 on the column-clipped lanes: raster -0.3 %, but the
// configs[4] SA trajectory changed, so some state's splats rely on it.)
#if defined(GGS_NO_RATIO_CLAMP) && GGS_NO_RATIO_CLAMP   // probe build only: does a parity test see it?
#define GGS_RATIO(qy8) GGS_EXP2(__builtin_fmaf((qy8), s.c128, abx.y))
#else
#define GGS_RATIO(qy8) GGS_EXP2(fminf(__builtin_fmaf((qy8), s.c128, abx.y), 100.0f))
#endif
// The first pair's exponent e = qy (Cc qy + bx) + px for both rows of the pair,
// as (qy/8) (64 Cc (qy/8) + 8 bx) + px (make_rec: the same bits).  64 Cc broadcast
// from the low half of the record's (C64, cx) SGPR pair, 8 bx from the high half
// of abx = (A qx, 8 Bc qx) and px from the low half of a VGPR pair whose
// high half is never set: no per-visit broadcast copies (LLVM copies a splat of a
// VGPR into a pair of its own; round 3: raster -0.2 % at 512^2, -0.5 % at 1024^2,
// bit-identical)
#define GGS_E1(qy) ({                                                                     \
        f2_t t_, e2_, pxu_;                                                               \
        pxu_.x = px;                                                                      \
        const uint64_t ccp_ = *reinterpret_cast<const uint64_t*>(&s.C64);                  \
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,1] op_sel_hi:[0,1,1]" : "=v"(t_) : "s"(ccp_), "v"(qy), "v"(abx)); \
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,1,0]" : "=v"(e2_) : "v"(qy), "v"(t_), "v"(pxu_)); \
        e2_; })
#define GGS_FOR8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define GGS_FOR16P(X) GGS_FOR8(X) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

// MODE: 0 = write image, 1 = fitness (weights from the target plan)
//
// One wave per workgroup (WPB); wave w of a 64 x TILE_H tile owns the
// 16-column strip [tx0+16w, tx0+16w+15] x TILE_H rows.  No workgroup barrier
// anywhere: each wave culls the candidate's splats against its own strip (64
// per step, highest index first, ballot + mbcnt compaction -> an order-
// preserving LDS list), blends that list front-to-back, and writes its own
// partial sum.  TILE_H = 128: 128 accumulator VGPRs (+~35) -> 3 waves per SIMD.
template <int MODE, bool SAT, bool FUSED>
__global__ void __launch_bounds__(GGS_DEPTH_SPLIT ? 2 * NT : NT, OCC)
raster_kernel(const SplatRec* __restrict__ recs, const int4* __restrict__ bnds, int B, int N, int H, int W, int nTX,
              int nTiles,
              float bg_r, float bg_g, float bg_b, float* __restrict__ img,
              const float4* __restrict__ plan, float* __restrict__ partials,
              const int* __restrict__ tile_order, const unsigned char* __restrict__ dirty,
              const float* __restrict__ clean, const int* __restrict__ live, int CH, FinFused fin, int simds) {
    constexpr bool DS = GGS_DEPTH_SPLIT && MODE == 1 && !SAT;
    // cull-list words carry the visit's scalar control (visit_word): the instances
    // without the saturation check and the folded finalize (in the GA's folded
    // instance they cost 3 SGPR spills to VGPR lanes; the saturation instances lost 1.5 %)
    constexpr bool VW = !SAT && !FUSED;
    __shared__ int lists[DS ? 2 : WPB][CAP];   // per-wave strip lists (descending splat index)

    const int lane = threadIdx.x & 63;
#if GGS_TIMING
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_cull = 0, t_vis = 0, t_mark = __builtin_amdgcn_s_memtime();
    unsigned n_vis = 0, n_done = 0;     // listed / blended visits
#endif
#if GGS_DEPTH_SPLIT
    const int wib = DS ? 0 : ufirst((int)(threadIdx.x >> 6));  // wave in block (uniform: keeps control on SALU)
    const int half = DS ? ufirst((int)(threadIdx.x >> 6)) : 0;  // depth split: 0 front, 1 back
#else
    const int wib = ufirst((int)(threadIdx.x >> 6));  // wave in block (uniform: keeps control on SALU)
#endif
    // SA loop rounds: the grid is sized for the session's capacity and only the
    // first *live candidates are evaluated; the grid order below is then that of
    // a launch over *live candidates, and the blocks past it exit at once
    if (live) {
        B = ufirst(*live);
        if ((int64_t)blockIdx.x >= (int64_t)B * nTiles * SPB) return;
    }
    // strip-major grid: B consecutive blocks run one strip (group) for every
    // candidate; groups go central (heavy) first to shorten the grid's tail.
    // Large launches run in candidate chunks of CH (all groups of one chunk, then
    // the next), so a chunk's records stay cached while its groups run
    int idx = blockIdx.x, b0 = 0, Bc = B;
    // A launch of 2-3 strip-waves per SIMD runs in one round: every wave is
    // resident from the start and the three sharing a SIMD (blocks r, r + S,
    // r + 2S, S = SIMDs) split its VALU, so the SIMD ends with the SUM of their
    // work (docs/EXPERIMENTS.md §14).  The middle third runs reversed: the
    // heaviest (central) strips then share a SIMD with the lightest of the
    // middle third instead of its heaviest (a boustrophedon over the expected
    // cost order; the bits do not depend on the order).  Shipped GA launch
    // (24 x 128 strips) raster -1.45 %; with two waves per SIMD (a lone 2048^2
    // SA neighbour) the pairing measured +1.05 %, so only above 2S (EXP §15)
    if (simds > 0) {
        const int n = B * nTiles * SPB;
        if (n > 2 * simds && n <= 3 * simds && idx >= simds && idx < 2 * simds) idx = 3 * simds - 1 - idx;
    }
    if (B > CH) {
        const int per = CH * nTiles * SPB;
        const int c = idx / per;
        idx -= c * per;
        b0 = c * CH;
        Bc = min(CH, B - b0);
    }
    const int gi = idx / Bc;
    const int grp = tile_order ? tile_order[gi] : gi;
    // candidates rotate by one per group: with B % 8 == 0 a fixed b would stay on
    // one XCD (blocks go round-robin to the 8 XCDs) and per-XCD work would be the
    // sum of 16 candidates' costs (tools/probe/wave_timing.py: XCD end times 197-207 us)
    // ... for the large-N instances only every 2^XCD_SHIFT groups: blocks B apart
    // (the next group's block in the same XCD slot) then run the same candidate,
    // whose records stay in that XCD's caches across 8 groups (see XCD_SHIFT)
    const int b = b0 + (int)((idx + (gi >> (SAT ? XCD_SHIFT : 0))) % Bc);
    const int t = grp / SPB;
    const int wv = (grp % SPB) * WPB + wib;           // strip 0..3 of the tile
    const int tx0 = (t % nTX) * TILE;
    const int ty0 = (t / nTX) * TILE_H;
    const int ty1 = min(ty0 + TILE_H, H) - 1;
    if (MODE != 0 && dirty) {         // incremental (SA): a strip no changed splat touches
        const int64_t slot = ((int64_t)b * nTiles + t) * 4 + wv;   // keeps the current state's
        if (!dirty[slot]) {                                         // partial, bit for bit
#if GGS_DEPTH_SPLIT
            if (DS && half) return;
#endif
            if (lane == 0) store_partial(partials + slot, clean[t * 4 + wv], FUSED);
            if (FUSED) strip_done(fin, partials, b, nTiles * 4, lane);
            return;
        }
    }

    const int sx0 = tx0 + wv * 16;    // this wave's strip: columns [sx0, sx0+15]
    const int col = sx0 + (lane & 15);
    const int ph = lane >> 4;         // row phase 0..3
    const float Xf = (float)col;
    const float Yb = (float)(ty0 + ph);
    // the lane's two rows of pair 0: a visit's first-pair offsets qy are one packed
    // subtract (round 3: -1.0 % raster vs qy0 then qy0 + 4)
    const f2_t Ybv = {0.125f * Yb, 0.125f * (Yb + 4.0f)};   // in eighths (see make_rec)

    // 16 pixels per lane x (R, G, B, transmittance), as named scalars: arrays
    // get vectorised into <16 x float> values whose phis the allocator splits.
#define GGS_DECL(k) f2_t P_R##k = 0.0f, P_G##k = 0.0f, P_B##k = 0.0f, P_T##k = 1.0f;
    GGS_FOR16P(GGS_DECL)
#undef GGS_DECL

    const SplatRec* __restrict__ crec = recs + (int64_t)b * N;
    const int4* __restrict__ cbnd = bnds + (int64_t)b * N;
#if GGS_DEPTH_SPLIT
    int* __restrict__ list = &lists[0][0] + (wib + half) * CAP;
    // the splat indices this wave culls: [nlo, nhi) (all of them but with the depth split)
    const int nlo = DS && half == 0 ? N / 2 : 0, nhi = DS && half == 1 ? N / 2 : N, nr = nhi - nlo;
    __shared__ int s_cnt[2];
    int lbase = 0, c0 = 0;            // depth split: this wave's part of the joint list
#define GGS_NHI nhi
#define GGS_NLO nlo
#define GGS_NR nr
#define GGS_LIST_AT(q) list_at(q)
#else
    int* __restrict__ list = &lists[0][0] + wib * CAP;
#define GGS_NHI N
#define GGS_NLO 0
#define GGS_NR N
#define GGS_LIST_AT(q) list[q]
#endif
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int cnt = 0;
    // every pixel of the strip below SAT_EPS transmittance (wave-uniform)
    auto saturated = [&]() __attribute__((always_inline)) {
        float m = 0.0f;
#define GGS_TMAX(k) if ((k) < NPK) m = fmaxf(m, fmaxf(P_T##k.x, P_T##k.y));
        GGS_FOR16P(GGS_TMAX)
#undef GGS_TMAX
        return !__ballot(m >= SAT_EPS);
    };

    // bounds of the next chunks are loaded ahead (the cull does little work per
    // chunk, so it waits on these loads): one chunk ahead at the bench's N (4 chunks
    // per strip; two: no gain there), two for the long saturation-cut culls, in two
    // registers the cull alternates, two chunks per step (a rotating copy, or a step
    // that may stop between the two, makes the compiler wait on the newest load)
    auto bounds = [&](int i) { return cbnd[max(i, 0)]; };
#ifndef GGS_CULL_AHEAD
#define GGS_CULL_AHEAD 2
#endif
    constexpr int AHEAD = SAT ? GGS_SAT_AHEAD : GGS_CULL_AHEAD;
    static_assert(AHEAD >= 1 && AHEAD <= 4, "cull prefetch depth");
    // issued in chunk order (sched barriers), so each chunk waits vmcnt(AHEAD - 1)
    int4 bbA = bounds(GGS_NHI - 1 - lane), bbB, bbC, bbD;
    if constexpr (AHEAD > 1) { __builtin_amdgcn_sched_barrier(0); bbB = bounds(GGS_NHI - 1 - lane - 64); }
    if constexpr (AHEAD > 2) { __builtin_amdgcn_sched_barrier(0); bbC = bounds(GGS_NHI - 1 - lane - 128); }
    if constexpr (AHEAD > 3) { __builtin_amdgcn_sched_barrier(0); bbD = bounds(GGS_NHI - 1 - lane - 192); }
    int base = 0;                     // first splat (from the back) not yet culled
    // a batch is handed to the blend once it holds more than LIMIT splats; a step
    // adds at most 64 * AHEAD, so the list (CAP) cannot overflow
    constexpr int LIMIT = SAT ? SAT_BATCH - 64 : CAP - 64 * AHEAD;
    static_assert(LIMIT + 64 * AHEAD <= CAP, "cull list capacity");
#if GGS_DEPTH_SPLIT
    // (the depth split: one pass, whose barrier both waves reach even with no splats)
    for (int pass = 0;; ++pass) {
        if (DS ? pass > 0 : base >= nr) break;
#else
    while (base < N) {
#endif
        // wave priority: the load-bound cull issues ahead of other waves' blends (+0.4 %)
        __builtin_amdgcn_s_setprio(CULL_PRIO);
        // --- cull 64 splats (descending index = front-to-back) against the strip:
        // one 16-B load per lane (clamped index, no short-circuit: a branchy test
        // splits it into two dependent loads), then a branch-free overlap test
#define GGS_CULL_CHUNK(BB)                                                                  \
        {                                                                                   \
            const int i = GGS_NHI - 1 - (base + lane);                                      \
            const int4 bb = BB;                                               /* x0 x1 y0 y1 */ \
            if (AHEAD == 1) BB = bounds(i - 64);                                            \
            const bool hit = (i >= GGS_NLO) & (bb.w >= ty0) & (bb.z <= ty1) & (bb.y >= sx0) & (bb.x <= sx0 + 15); \
            /* deeper: reload after the test, into the registers just read */              \
            if (AHEAD > 1) BB = bounds(i - 64 * AHEAD);                                     \
            const uint64_t m = __ballot(hit);                                               \
            if (hit) list[cnt + __popcll(m & lt_mask)] =                                    \
                VW ? visit_word(i, bb, ty0, sx0) : i * (int)sizeof(SplatRec);                \
            cnt += __popcll(m);                                                             \
            base += 64;                                                                     \
        }
        if constexpr (AHEAD == 1) {
            GGS_CULL_CHUNK(bbA)
            if (cnt <= LIMIT && base < GGS_NR) continue;
        } else {
            do {                                  // past N: no hits (i < 0), clamped loads
                GGS_CULL_CHUNK(bbA)
                GGS_CULL_CHUNK(bbB)
                if constexpr (AHEAD > 2) GGS_CULL_CHUNK(bbC)
                if constexpr (AHEAD > 3) GGS_CULL_CHUNK(bbD)
            } while (cnt <= LIMIT && base < GGS_NR);
        }
#undef GGS_CULL_CHUNK
#if GGS_DEPTH_SPLIT
        if constexpr (DS) {           // N / 2 <= SAT_MIN_SPLATS / 2 < LIMIT: culled in one batch
            static_assert(!DS || SAT_MIN_SPLATS / 2 + 64 * AHEAD <= CAP, "depth split: one cull batch");
            if (lane == 0) s_cnt[half] = cnt;
            __syncthreads();
            c0 = ufirst(s_cnt[0]);
            const int total = c0 + ufirst(s_cnt[1]), hs = (total + 1) >> 1;
            lbase = half ? hs : 0;
            cnt = half ? total - hs : hs;
        }
#endif
        if (cnt == 0) continue;       // (base >= N: the loop ends)
        __builtin_amdgcn_s_setprio(0);
#if GGS_TIMING
        { GGS_TMARK(now); t_cull += now - t_mark; t_mark = now; n_vis += cnt; }
#endif

        // --- blend the list: splat params arrive in SGPRs (s_load), the next
        //     record is fetched while the current one is blended; list indices
        //     are read 64 at a time into a VGPR (one per lane) and picked with
        //     v_readlane, so no LDS latency sits on the per-splat path ---------
        // (byte offsets: the record load takes the readlane result as its
        //  32-bit SGPR offset; past the list end it reloads a listed record)
        const char* __restrict__ cbase = reinterpret_cast<const char*>(crec);
#if GGS_DEPTH_SPLIT
        // the joint list of the depth split: lists[0][0, c0) then lists[1]
        auto list_at = [&](int q) __attribute__((always_inline)) {
            if constexpr (DS) {
                q += lbase;
                const int a0 = lists[0][min(q, CAP - 1)], a1 = lists[1][max(q - c0, 0)];
                return q < c0 ? a0 : a1;
            } else {
                return list[q];
            }
        };
#endif
        int offv = GGS_LIST_AT(min(lane, cnt - 1));
        // one (splat, strip) visit: cull-list record s (list word w) -> the strip's accumulators
        auto visit = [&](const SplatRec& s, const unsigned w) __attribute__((always_inline)) {
#if GGS_TIMING
            ++n_done;
#endif
            const int x0 = s.x0, x1 = s.x1, y0 = s.y0, y1 = s.y1;
            const int dy0 = y0 - ty0, dy1 = y1 - ty0;          // AABB rows relative to the tile
            const int gA = max(dy0, 0) >> 2;                   // first / last row group
            const int gB = min(dy1, TILE_H - 1) >> 2;
            const float qx = Xf - s.cx;
            f2_t abx;                          // (A qx, 8 Bc qx): one v_pk_mul from the (A, B8) pair
            abx.x = s.A * qx;
            abx.y = s.B8 * qx;
            float px = __builtin_fmaf(abx.x, qx, s.la);
            // the AABB's column clip: only when it cuts the strip's 16 columns (a
            // wave-uniform branch; 85 % of the bench's visits span all 16 columns.
            // The empty asm keeps the compiler from if-converting it back into an
            // unconditional compare + select).  Dead lanes: px = -inf (f = 0; the
            // ratio's clamp keeps their walk at 0, see GGS_RATIO).
            if (__builtin_expect(VW ? (w >> VW_CLIP) != 0 : max(x0 - sx0, sx0 + 15 - x1) > 0, 0)) {
                const bool inx = (unsigned)(col - x0) <= (unsigned)(x1 - x0);
                px = inx ? px : -__builtin_inff();
                asm volatile("" : "+v"(px));
            }
            const f2_t qyv = Ybv - (f2_t)s.cy8;          // qy / 8 of the lane's rows
            const int rlo = y0 - ty0 - ph;                     // row test: 4g - rlo in [0, rspan]
            const unsigned rspan = (unsigned)(y1 - y0);

            // first / last group pair; kB = NPK: the splat reaches past the tile's
            // last row, so the walk's last pair needs no bottom-row mask (about half
            // the partial visits: 4 VALU fewer each, the same bits)
            // the visit's scalar control: from the list word, or (saturation instances) here
            const int kA = VW ? (int)(w >> VW_KA) & 15 : gA >> 1;
            const int kB = VW ? (int)w & 31 : (dy1 >= TILE_H - 1 ? NPK : gB >> 1);
            f2_t F2, R2;                                       // row recurrence: f, ratio
            // First pair: exact exponent; keeps the unmasked f as the recurrence
            // seed and, when more pairs follow, the ratio 2^d to the next pair.
            // A seed below 2^-100 (0x0D800000) on a live lane (tiny corner of a thin rotated
            // splat) would lose the recurrence's precision: that wave walks this
            // splat with the exact exponent instead (wave-uniform, ~0.3 % of walks).
            // Full-height visits (the splat spans the strip's 128 rows: ~45 % of
            // them on the bench population) need no row mask and no walk exit
            // test: one straight-line block, the same arithmetic as the general
            // walk (kA = 0, kB = NPK-1, all-ones masks), so the same bits.
            if (VW ? (w & 63u) == (VW_ABOVE | NPK) : max(dy0, TILE_H - 1 - dy1) <= 0) {   // y0 <= ty0, y1 >= ty0 + 127
                const f2_t e_ = GGS_E1(qyv);
                F2.x = GGS_EXP2(e_.x);
                F2.y = GGS_EXP2(e_.y);
                if ((__float_as_uint(s.rho4) >> 31) &&          // only flagged splats (make_rec)
                    __ballot((px > -__builtin_inff()) &
                             (min(__float_as_uint(F2.x), __float_as_uint(F2.y)) < 0x0D800000u))) {
                    GGS_BLEND(0, F2);
                    goto x0;
                }
                GGS_BLEND(0, F2);
                // d(qy) = 16 Cc (qy + 4) + 8 bx; the .y row's ratio is 2^(64 Cc) times it
                R2.x = GGS_RATIO(qyv.y);
                R2.y = R2.x * __builtin_fabsf(s.rho4);
#define GGS_FULL(k)                                                                     \
    if ((k) >= 1 && (k) < NPK - 1) {                                                    \
        GGS_BLEND_REC(k)                                                                \
    } else if ((k) == NPK - 1) {      /* last pair: no ratio update */                  \
        F2 = F2 * R2;                                                                   \
        GGS_BLEND(k, F2);                                                               \
    }
                GGS_FOR16P(GGS_FULL)
#undef GGS_FULL
                goto done;
            }
            // About half the partial visits start above the tile (the splat began in
            // a tile above): their first pair needs no top-row mask (GGS_FIRST(0)
            // with all-ones masks: the same bits, 4 VALU fewer).
            if (VW ? (w & VW_ABOVE) != 0 : dy0 <= 0) {        // dy0 <= 0
                const f2_t e_ = GGS_E1(qyv);
                F2.x = GGS_EXP2(e_.x);
                F2.y = GGS_EXP2(e_.y);
                if (kB == 0) {                                 // one pair: bottom limit only
                    const PairLanes bot_ = rows_upto(dy1);
                    f2_t fu_;
                    fu_.x = keep_if(bot_.x, F2.x);
                    fu_.y = keep_if(bot_.y, F2.y);
                    GGS_BLEND(0, fu_);
                    goto done;
                }
                GGS_BLEND(0, F2);
                if ((__float_as_uint(s.rho4) >> 31) &&
                    __ballot((px > -__builtin_inff()) &
                             (min(__float_as_uint(F2.x), __float_as_uint(F2.y)) < 0x0D800000u)))
                    goto x0;
                R2.x = GGS_RATIO(qyv.y);
                R2.y = R2.x * __builtin_fabsf(s.rho4);
                goto u0;
            }
            // the rest of the visits starting in pair 0: before the switch's compare tree
            if (kA == 0) goto f0;
            switch (kA) {
#define GGS_FIRST(k)                                                                    \
    case k:                                                                             \
    f##k: __attribute__((unused));                                                      \
        if (k < NPK) {                                                                  \
            const f2_t qy_ = (k) == 0 ? qyv : qyv + (f2_t)(float)(k);                   \
            const f2_t e_ = GGS_E1(qy_);                                                \
            F2.x = GGS_EXP2(e_.x);                                                      \
            F2.y = GGS_EXP2(e_.y);                                                      \
            f2_t fu_;                                                                   \
            const PairLanes top_ = rows_from(y0 - ty0 - 8 * (k));                       \
            if (kB == k) {                /* one pair: both AABB row limits */          \
                const PairLanes bot_ = rows_upto(y1 - ty0 - 8 * (k));                   \
                fu_.x = keep_if(top_.x & bot_.x, F2.x);                                 \
                fu_.y = keep_if(top_.y & bot_.y, F2.y);                                 \
                GGS_BLEND(k, fu_);                                                      \
                goto done;                                                              \
            }                                                                           \
            fu_.x = keep_if(top_.x, F2.x);                                              \
            fu_.y = keep_if(top_.y, F2.y);                                              \
            GGS_BLEND(k, fu_);                                                          \
            /* guard on the seed's bits (f >= 0: unsigned order = float order);  */     \
            /* dead lanes (px = -inf) excluded                                    */     \
            if ((__float_as_uint(s.rho4) >> 31) &&                                      \
                __ballot((px > -__builtin_inff()) &                                     \
                         (min(__float_as_uint(F2.x), __float_as_uint(F2.y)) < 0x0D800000u))) \
                goto x##k;                                                              \
            /* d(qy) = 16 Cc (qy + 4) + 8 bx, the .y row's ratio 2^(64 Cc) times */     \
            R2.x = GGS_RATIO(qy_.y);                                                    \
            R2.y = R2.x * __builtin_fabsf(s.rho4);                                      \
            goto u##k;                                                                  \
        }                                                                               \
        break;
                GGS_FIRST(0) GGS_FIRST(1) GGS_FIRST(2) GGS_FIRST(3) GGS_FIRST(4)
                GGS_FIRST(5) GGS_FIRST(6) GGS_FIRST(7) GGS_FIRST(8) GGS_FIRST(9)
                GGS_FIRST(10) GGS_FIRST(11) GGS_FIRST(12) GGS_FIRST(13) GGS_FIRST(14)
                GGS_FIRST(15)
#undef GGS_FIRST
                default: __builtin_unreachable();
            }
            // recurrence walk: f *= r, r *= rho (no exp).  Three pairs per basic
            // block (the walk's scalar branches split blocks), so the scheduler
            // overlaps one pair's blend with the next pairs' recurrence (round 3:
            // -0.6 % at 512^2, -0.3 % at 1024^2 vs two; four: a further -0.2 %).
            // The last pair (rows below y1 masked) is inlined at every exit of
            // each step, so leaving the walk costs no second switch.
#define GGS_LASTB(k)                                                                    \
    if ((k) < NPK) {                                                                    \
        const f2_t fr_ = F2 * R2;                                                       \
        const PairLanes bot_ = rows_upto(y1 - ty0 - 8 * (k));                           \
        f2_t fu_;                                                                       \
        fu_.x = keep_if(bot_.x, fr_.x);                                                 \
        fu_.y = keep_if(bot_.y, fr_.y);                                                 \
        GGS_BLEND(k, fu_);                                                              \
    }
// the tile's last pair when the splat reaches past it (kB == NPK): no mask
#define GGS_LASTF(k)                                                                    \
    if ((k) < NPK) {                                                                    \
        F2 = F2 * R2;                                                                   \
        GGS_BLEND(k, F2);                                                               \
    }
#define GGS_MID3(k, k1, k2, k3)                                                         \
    u##k:                                                                               \
        if (__builtin_expect(kB > (k3), 1)) {                                           \
            GGS_BLEND_REC(k1) GGS_BLEND_REC(k2)                                         \
            if ((k3) == NPK - 1) {                                                      \
                GGS_LASTF(k3)                                                           \
                goto done;                                                              \
            }                                                                           \
            GGS_BLEND_REC(k3)                                                           \
            goto u##k3;                                                                 \
        }                                                                               \
        if (kB == (k3)) {                                                               \
            GGS_BLEND_REC(k1) GGS_BLEND_REC(k2)                                         \
            GGS_LASTB(k3)                                                               \
            goto done;                                                                  \
        }                                                                               \
        if (kB == (k2)) {                                                               \
            GGS_BLEND_REC(k1)                                                           \
            GGS_LASTB(k2)                                                               \
            goto done;                                                                  \
        }                                                                               \
        GGS_LASTB(k1)                                                                   \
        goto done;
            // laid out as three chains (u0 u3 u6 u9 u12 u15, u1 u4 ... u13, u2 u5 ...
            // u14), so a walk continuing past its step falls through into the next
            // step instead of taking a branch every three pairs
            GGS_MID3(0, 1, 2, 3) GGS_MID3(3, 4, 5, 6) GGS_MID3(6, 7, 8, 9) GGS_MID3(9, 10, 11, 12)
            GGS_MID3(12, 13, 14, 15)
        u15:
            goto done;
            GGS_MID3(1, 2, 3, 4) GGS_MID3(4, 5, 6, 7) GGS_MID3(7, 8, 9, 10) GGS_MID3(10, 11, 12, 13)
        u13:                          // pairs 14 and 15 are the last ones there are
            if (kB == NPK) {
                GGS_BLEND_REC(14)
                GGS_LASTF(15)
                goto done;
            }
            if (kB == 15) {
                GGS_BLEND_REC(14)
                GGS_LASTB(15)
                goto done;
            }
            GGS_LASTB(14)
            goto done;
            GGS_MID3(2, 3, 4, 5) GGS_MID3(5, 6, 7, 8) GGS_MID3(8, 9, 10, 11) GGS_MID3(11, 12, 13, 14)
        u14:
            if (kB == NPK) {
                GGS_LASTF(15)
                goto done;
            }
            GGS_LASTB(15)
            goto done;
#undef GGS_MID3
#undef GGS_LASTB
#undef GGS_LASTF
            // exact walk (guard tripped): the exponent per pair as before
#define GGS_XMID(kp, k) x##kp: if (kB == k) goto xlast; if (k < NPK) GGS_PK(k, false);
            GGS_XMID(0, 1) GGS_XMID(1, 2) GGS_XMID(2, 3) GGS_XMID(3, 4) GGS_XMID(4, 5)
            GGS_XMID(5, 6) GGS_XMID(6, 7) GGS_XMID(7, 8) GGS_XMID(8, 9) GGS_XMID(9, 10)
            GGS_XMID(10, 11) GGS_XMID(11, 12) GGS_XMID(12, 13) GGS_XMID(13, 14)
            GGS_XMID(14, 15)
#undef GGS_XMID
        x15:
        xlast:
            switch (kB == NPK ? 16 : kB) {   // (case 16: pair NPK-1 ran unmasked)
#define GGS_LAST(k) case k: if (k < NPK) GGS_PK(k, true); break;
                GGS_LAST(1) GGS_LAST(2) GGS_LAST(3) GGS_LAST(4) GGS_LAST(5) GGS_LAST(6)
                GGS_LAST(7) GGS_LAST(8) GGS_LAST(9) GGS_LAST(10) GGS_LAST(11) GGS_LAST(12)
                GGS_LAST(13) GGS_LAST(14) GGS_LAST(15)
                case 16: break;               // kB == NPK: the last pair ran unmasked
#undef GGS_LAST
                default: __builtin_unreachable();
            }
        done:;
        };
#undef rows_from
#undef rows_upto
        // two records in alternating SGPR sets: the next record is loaded into
        // the set the finished visit used, so no register rotation at the latch
        auto word_at = [&](int jj) __attribute__((always_inline)) {
            return (unsigned)__builtin_amdgcn_readlane(offv, jj & 63);
        };
        auto load_at = [&](unsigned w) __attribute__((always_inline)) {
            return *reinterpret_cast<const SplatRec*>(cbase + (VW ? (w & VW_OFFSET) : w));
        };
        unsigned wa = word_at(0);
        SplatRec ra = load_at(wa);
        int jr = 63;                  // last j before the next 64 offsets are needed
        for (int j = 0;;) {
            if (__builtin_expect(j == jr, 0)) { jr += 64; offv = GGS_LIST_AT(min(j + 1 + lane, cnt - 1)); }
            const unsigned wb = word_at(j + 1);
            const SplatRec rb = load_at(wb);
            visit(ra, wa);
            if (++j >= cnt) break;
            if (__builtin_expect(j == jr, 0)) { jr += 64; offv = GGS_LIST_AT(min(j + 1 + lane, cnt - 1)); }
            wa = word_at(j + 1);
            ra = load_at(wa);
            visit(rb, wb);
            if (++j >= cnt) break;
#if GGS_SATURATE
            // (strips reaching past the image keep T = 1 outside it: never cut)
            if (SAT && j >= SAT_FIRST && (j & (SAT_EVERY - 1)) == 0 && sx0 + 15 < W && ty0 + TILE_H <= H) {
                if (saturated()) {   // skip the rest of the list and of the cull
                    base = N;
                    break;
                }
            }
#endif
        }
#if GGS_SATURATE
        // end of a batch with more splats to cull: stop here if the strip is saturated
        if (SAT && SAT_BATCH < CAP && base < N && sx0 + 15 < W && ty0 + TILE_H <= H && saturated())
            base = N;
#endif
        cnt = 0;
#if GGS_TIMING
        { GGS_TMARK(now); t_vis += now - t_mark; t_mark = now; }
#endif
    }

#undef GGS_NHI
#undef GGS_NLO
#undef GGS_NR
#undef GGS_LIST_AT
#if GGS_DEPTH_SPLIT
    if constexpr (DS) {
        // wave 1 hands its (C, T) to wave 0 through the lists' 8 KB, four pairs
        // (32 floats per lane) at a time; wave 0 composes front over back
        float* __restrict__ xs = reinterpret_cast<float*>(&lists[0][0]);
        __syncthreads();              // both waves done with the lists
#define GGS_XW(k, k0)                                                                  \
        if ((k) < NPK) {                                                               \
            float* x_ = xs + 8 * ((k) - (k0)) * 64 + lane;                             \
            x_[0] = P_R##k.x; x_[64] = P_R##k.y; x_[128] = P_G##k.x; x_[192] = P_G##k.y;   \
            x_[256] = P_B##k.x; x_[320] = P_B##k.y; x_[384] = P_T##k.x; x_[448] = P_T##k.y; \
        }
#define GGS_XR(k, k0)                                                                  \
        if ((k) < NPK) {                                                               \
            const float* x_ = xs + 8 * ((k) - (k0)) * 64 + lane;                       \
            const f2_t rb_ = {x_[0], x_[64]}, gb_ = {x_[128], x_[192]};                \
            const f2_t bb_ = {x_[256], x_[320]}, tb_ = {x_[384], x_[448]};             \
            P_R##k = fma2(P_T##k, rb_, P_R##k);                                        \
            P_G##k = fma2(P_T##k, gb_, P_G##k);                                        \
            P_B##k = fma2(P_T##k, bb_, P_B##k);                                        \
            P_T##k = P_T##k * tb_;                                                     \
        }
#define GGS_XCHUNK(k0, k1, k2, k3)                                                     \
        if (half) { GGS_XW(k0, k0) GGS_XW(k1, k0) GGS_XW(k2, k0) GGS_XW(k3, k0) }      \
        __syncthreads();                                                               \
        if (!half) { GGS_XR(k0, k0) GGS_XR(k1, k0) GGS_XR(k2, k0) GGS_XR(k3, k0) }      \
        __syncthreads();
        GGS_XCHUNK(0, 1, 2, 3) GGS_XCHUNK(4, 5, 6, 7) GGS_XCHUNK(8, 9, 10, 11) GGS_XCHUNK(12, 13, 14, 15)
#undef GGS_XCHUNK
#undef GGS_XR
#undef GGS_XW
        if (half) return;
    }
#endif

    // --- epilogue ---------------------------------------------------------------
    float R[RG], G[RG], Bl[RG], T[RG];
#define GGS_PACK(k)                                                                   \
    if (k < NPK) {                                                                    \
        R[2 * k] = P_R##k.x; G[2 * k] = P_G##k.x; Bl[2 * k] = P_B##k.x; T[2 * k] = P_T##k.x; \
        R[2 * k + 1] = P_R##k.y; G[2 * k + 1] = P_G##k.y; Bl[2 * k + 1] = P_B##k.y;   \
        T[2 * k + 1] = P_T##k.y;                                                      \
    }
    GGS_FOR16P(GGS_PACK)
#undef GGS_PACK
    if (MODE == 0) {
        if (col < W) {
#pragma unroll
            for (int g = 0; g < RG; ++g) {
                const int row = ty0 + 4 * g + ph;
                if (row < H) {
                    // streaming (non-temporal) stores: the image is never re-read by this
                    // launch, and write-allocating 384 MiB per 512^2/128 launch in L2
                    // evicts the records and cull bounds every strip-wave re-reads
                    float* o = img + (((int64_t)b * H + row) * W + col) * 3;
                    __builtin_nontemporal_store(fminf(fmaxf(__builtin_fmaf(T[g], bg_r, R[g]), 0.0f), 1.0f), o + 0);
                    __builtin_nontemporal_store(fminf(fmaxf(__builtin_fmaf(T[g], bg_g, G[g]), 0.0f), 1.0f), o + 1);
                    __builtin_nontemporal_store(fminf(fmaxf(__builtin_fmaf(T[g], bg_b, Bl[g]), 0.0f), 1.0f), o + 2);
                }
            }
        }
    } else {
        // The target plan (plan_kernel) holds, per lane and row-group pair
        // (g, g+1) = (2k, 2k+1), two float4s: (t_r, t_r', t_g, t_g') and
        // (t_b, t_b', w, w'), w already mode-specific and 0 outside the image:
        // coalesced 16-B loads, no address math, no bounds tests, and the pair
        // lines up with the packed accumulators (two pixels per v_pk op).
        const float4* __restrict__ P = plan + (int64_t)(t * 4 + wv) * RG * 64 + lane;
        f2_t accp = 0.0f;
        // background pairs (bg, bg) in SGPR pairs: no VGPRs at the epilogue's peak
        const uint64_t bg2r = (uint64_t)__float_as_uint(bg_r) * 0x100000001ull;
        const uint64_t bg2g = (uint64_t)__float_as_uint(bg_g) * 0x100000001ull;
        const uint64_t bg2b = (uint64_t)__float_as_uint(bg_b) * 0x100000001ull;
#pragma unroll
        for (int k = 0; k < NPK; ++k) {
#if GGS_NOPLAN     // traffic probe only (wrong fitness): the epilogue reads no plan
            const float4 qa = make_float4(0.5f, 0.5f, 0.5f, 0.5f), qb = qa;
#else
            const float4 qa = P[(2 * k) * 64], qb = P[(2 * k + 1) * 64];
#endif
            // packed: one v_pk_fma_f32 with the clamp bit per channel and row pair
            // (the compiler folds the clamp only into the scalar v_fma_f32)
            const f2_t T2 = {T[2 * k], T[2 * k + 1]};
            f2_t c_r, c_g, c_b;
            asm("v_pk_fma_f32 %0, %1, %2, %3 clamp" : "=v"(c_r) : "v"(T2), "s"(bg2r), "v"((f2_t){R[2 * k], R[2 * k + 1]}));
            asm("v_pk_fma_f32 %0, %1, %2, %3 clamp" : "=v"(c_g) : "v"(T2), "s"(bg2g), "v"((f2_t){G[2 * k], G[2 * k + 1]}));
            asm("v_pk_fma_f32 %0, %1, %2, %3 clamp" : "=v"(c_b) : "v"(T2), "s"(bg2b), "v"((f2_t){Bl[2 * k], Bl[2 * k + 1]}));
            const f2_t dr = c_r - (f2_t){qa.x, qa.y};
            const f2_t dg = c_g - (f2_t){qa.z, qa.w};
            const f2_t db = c_b - (f2_t){qb.x, qb.y};
            const f2_t d2 = fma2(dr, dr, fma2(dg, dg, db * db));
            accp = fma2((f2_t){qb.z, qb.w}, d2, accp);
        }
        float acc = accp.x + accp.y;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0)        // one partial per (candidate, tile, strip): no block barrier
            store_partial(partials + ((int64_t)b * nTiles + t) * 4 + wv, acc, FUSED);
        if (FUSED) strip_done(fin, partials, b, nTiles * 4, lane);
    }
#if GGS_TIMING
    {
        GGS_TMARK(now);
        const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();
        if (lane == 0 && blockIdx.x < GGS_TIMING_WAVES) {
            unsigned long long* o = g_ggs_timing + 8 * (size_t)blockIdx.x;
            o[0] = rt_start; o[1] = rt_end; o[2] = t_cull; o[3] = t_vis; o[4] = now - t_mark;
            o[5] = (unsigned long long)__builtin_amdgcn_s_getreg(0xF804) |
                   ((unsigned long long)__builtin_amdgcn_s_getreg(0xF814) << 32);
            o[6] = n_vis; o[7] = n_done;
        }
    }
#endif
}

// ---------------------------------------------------------------------------
// target plan: the fitness epilogue's inputs re-laid out in raster lane order
// ---------------------------------------------------------------------------
// Four waves per (tile, strip), PLAN_KP row-group pairs each (loads unrolled:
// one wave per strip walking all 16 pairs was a chain of dependent HBM round
// trips, 23 us at 512^2).  For the row-group pair (2k, 2k+1) of the pixel
// column this lane owns: plan[((t*4 + strip)*RG + 2k)*64 + lane] =
// (t_r, t_r', t_g, t_g') and [... + 2k+1] = (t_b, t_b', w, w') (primed: row
// group 2k+1), the raster epilogue's packed order; w is the pixel weight of
// fitness.py:17-31 for the mode (1 / mask / 1+beta*clamp(mask)) and 0 outside
// the image.  Each wave's sum of w goes to the weight block (plan_wsum_kernel
// reduces them to the plan's Sum w, a double).  Target and mask are constant
// over a GA run, so the plan is built once per (target, mask, mode, beta).
constexpr int PLAN_Q = 4, PLAN_KP = RG / 2 / PLAN_Q;
__global__ void __launch_bounds__(64)
plan_kernel(const float* __restrict__ target, const float* __restrict__ mask, int mode, float beta,
            int H, int W, int nTX, float4* __restrict__ plan, float* __restrict__ wave_w) {
    const int lane = threadIdx.x;
    const int sg = blockIdx.x / PLAN_Q, q = blockIdx.x % PLAN_Q;     // strip (t*4 + wv), quarter
    const int t = sg >> 2, wv = sg & 3;
    const int tx0 = (t % nTX) * TILE, ty0 = (t / nTX) * TILE_H;
    const int col = tx0 + wv * 16 + (lane & 15), ph = lane >> 4;
    float4* __restrict__ P = plan + (int64_t)sg * RG * 64 + lane;
    float wacc = 0.0f;
#pragma unroll
    for (int kk = 0; kk < PLAN_KP; ++kk) {
        const int k = q * PLAN_KP + kk;
        float tr[2], tg[2], tb[2], wg[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = ty0 + 4 * (2 * k + h) + ph;
            const bool ok = (row < H) & (col < W);
            const int64_t p = (int64_t)min(row, H - 1) * W + min(col, W - 1);
            float wgt = 1.0f;
            if (mode == GGS_FIT_WEIGHTED) wgt = mask[p];
            if (mode == GGS_FIT_BOOST) wgt = 1.0f + beta * fminf(fmaxf(mask[p], 0.0f), 1.0f);
            wgt = ok ? wgt : 0.0f;
            tr[h] = target[p * 3 + 0]; tg[h] = target[p * 3 + 1]; tb[h] = target[p * 3 + 2];
            wg[h] = wgt;
            wacc += wgt;
        }
        P[(2 * k) * 64] = make_float4(tr[0], tr[1], tg[0], tg[1]);
        P[(2 * k + 1) * 64] = make_float4(tb[0], tb[1], wg[0], wg[1]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wacc += __shfl_xor(wacc, o);
    if (lane == 0) wave_w[blockIdx.x] = wacc;
}

// Sum w of the plan in float64, fixed order (lane-strided, then the xor
// butterfly of wave_sum): the weighted / boost modes' denominator
// (fitness.py:23-31), once per plan instead of once per candidate.
__global__ void __launch_bounds__(64)
plan_wsum_kernel(const float* __restrict__ wave_w, int n, double* __restrict__ wsum) {
    const double v = wave_sum(wave_w, n);
    if (threadIdx.x == 0) *wsum = v;
}

hipError_t launch_plan(hipStream_t st, const float* target, const float* mask, int mode, float beta,
                       int H, int W, float4* plan, float* wblock) {
    int nTX;
    const int nTiles = raster_tiles(H, W, &nTX);
    const int nw = nTiles * 4 * PLAN_Q;
    float* wave_w = wblock + 4;                  // after the double (16-B slot)
    hipLaunchKernelGGL(plan_kernel, dim3(nw), dim3(64), 0, st, target, mask, mode, beta, H, W, nTX, plan, wave_w);
    hipLaunchKernelGGL(plan_wsum_kernel, dim3(1), dim3(64), 0, st, wave_w, nw, reinterpret_cast<double*>(wblock));
    return hipGetLastError();
}

size_t plan_wsum_bytes(int H, int W) { return 16 + sizeof(float) * 4 * PLAN_Q * (size_t)raster_tiles(H, W, nullptr); }

// ---------------------------------------------------------------------------
// dirty strips (incremental SA evaluation, SURVEY.md §8f #4 / annealing.py:121-146)
// ---------------------------------------------------------------------------
// Thread per (neighbour b, splat i): if the splat changed, every strip its old or
// new AABB touches is marked dirty for neighbour b.  Strips no changed splat
// touches keep their cull list and blend order, so their partial is the current
// state's.  "Changed" (rule): 1 = its 64-B raster record differs (the record holds
// everything the raster reads of a splat, its AABB included, so an unchanged
// record cannot move any strip's bits; a theta moved by an ulp by the double
// wrap_angle of genetic.py:71 + utils.py:43 often leaves the record as it was);
// 0 = any of its 9 genes differ bitwise (the round-2 rule).
__device__ __forceinline__ void mark_strips(const SplatRec& r, int nTX, unsigned char* __restrict__ d) {
    for (int ty = r.y0 / TILE_H; ty <= r.y1 / TILE_H; ++ty)
        for (int sx = r.x0 / 16; sx <= r.x1 / 16; ++sx) d[(ty * nTX + (sx >> 2)) * 4 + (sx & 3)] = 1;
}

__global__ void __launch_bounds__(256)
dirty_kernel(const float* __restrict__ curr, const float* __restrict__ nb,
             const SplatRec* __restrict__ cur_recs, const SplatRec* __restrict__ nb_recs, int n, int N,
             int nTX, int nTiles, unsigned char* __restrict__ dirty, unsigned* __restrict__ n_changed,
             const int* __restrict__ live, int rule) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)(live ? min(*live, n) : n) * N) return;
    const int b = (int)(idx / N), i = (int)(idx % N);
    unsigned diff = 0;
    if (rule == 1) {
        const uint4* a = reinterpret_cast<const uint4*>(cur_recs + i);
        const uint4* c = reinterpret_cast<const uint4*>(nb_recs + idx);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 x = a[k], y = c[k];
            diff |= (x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w);
        }
    } else {
        const unsigned* a = reinterpret_cast<const unsigned*>(curr + (int64_t)i * 9);
        const unsigned* c = reinterpret_cast<const unsigned*>(nb + idx * 9);
#pragma unroll
        for (int k = 0; k < 9; ++k) diff |= a[k] ^ c[k];
    }
    if (!diff) return;
    unsigned char* d = dirty + (int64_t)b * nTiles * 4;
    mark_strips(cur_recs[i], nTX, d);
    mark_strips(nb_recs[idx], nTX, d);
    if (n_changed) atomicAdd(n_changed, 1u);
}

hipError_t launch_dirty(hipStream_t st, const float* curr, const float* nb, const SplatRec* cur_recs,
                        const SplatRec* nb_recs, int n, int N, int H, int W, unsigned char* dirty,
                        unsigned* n_changed, const int* live, int rule) {
    int nTX;
    const int nTiles = raster_tiles(H, W, &nTX);
    hipError_t e = hipMemsetAsync(dirty, 0, (size_t)n * nTiles * 4, st);
    if (e != hipSuccess) return e;
    const int64_t tot = (int64_t)n * N;
    if (tot == 0) return hipSuccess;
    hipLaunchKernelGGL(dirty_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, curr, nb,
                       cur_recs, nb_recs, n, N, nTX, nTiles, dirty, n_changed, live, rule);
    return hipGetLastError();
}

size_t plan_bytes(int H, int W) { return sizeof(float4) * 4 * (size_t)raster_tiles(H, W, nullptr) * RG * 64; }

// ---------------------------------------------------------------------------
// finalize: fixed-order float64 reduction of tile partials -> fitness scalar
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
finalize_kernel(const float* __restrict__ partials, const float* __restrict__ wpartials,
                int nTiles, int mode, double hw, int B, float* __restrict__ out, const int* __restrict__ live) {
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);   // one wave per candidate (ggs_prep.h)
    if (b >= B || (live && b >= *live)) return;
    const float v = finalize_wave(partials, wpartials, nTiles, mode, hw, b);
    if ((threadIdx.x & 63) == 0) out[b] = v;
}

// ---------------------------------------------------------------------------
// detmath probe (parity tests of the deterministic functions, ggs_detmath_eval)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
detmath_kernel(const float* __restrict__ x, const float* __restrict__ y, int64_t n, int fn,
               float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float a = x[i];
    float r, s, c;
    switch (fn) {
        case 0: r = det_expf(a); break;
        case 1: r = det_logf(a); break;
        case 2: det_sincosf(a, &s, &c); r = s; break;
        case 3: det_sincosf(a, &s, &c); r = c; break;
        case 4: r = ggs_sqrt_rn(a); break;
        default: r = ggs_div_rn(a, y[i]); break;
    }
    out[i] = r;
}

hipError_t launch_detmath(hipStream_t st, const float* x, const float* y, int64_t n, int fn,
                          float* out) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(detmath_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, y, n,
                       fn, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// launchers (called from ggs_capi.cpp; no allocation, no sync)
// ---------------------------------------------------------------------------
hipError_t launch_prep(hipStream_t st, bool encode, const float* genomes, int64_t S, int C, int H,
                       int W, float k, SplatRec* recs, int4* bnds, float* f9, int* i4, float* enc9, const int* live,
                       int n_per) {
    if (S <= 0) return hipSuccess;
    constexpr int PB = 256;           // 64-thread blocks (all CUs busy): no change, round 3
    const unsigned grid = (unsigned)((S + PB - 1) / PB);
    if (encode)
        hipLaunchKernelGGL(prep_kernel<true>, dim3(grid), dim3(PB), 0, st, genomes, S, C, H, W, k,
                           recs, bnds, f9, i4, enc9, live, n_per);
    else
        hipLaunchKernelGGL(prep_kernel<false>, dim3(grid), dim3(PB), 0, st, genomes, S, C, H, W, k,
                           recs, bnds, f9, i4, enc9, live, n_per);
    return hipGetLastError();
}

// Dispatch order of the (tile, block-in-tile) groups: nearest the canvas
// centre first.  Splat density, and so a strip's cull list, peaks in the middle
// (AABBs are clipped at the borders); running the long strips first leaves the
// short ones to fill the grid's last round (list-scheduling model of the bench
// population: 1.135x -> 1.098x the ideal makespan; tile-granular order 1.135x).
void raster_tile_order(int H, int W, int* order) {
    int nTX;
    const int n = raster_tiles(H, W, &nTX) * SPB;
    std::vector<std::pair<double, int>> d(n);
    for (int g = 0; g < n; ++g) {
        const int t = g / SPB, s = g % SPB;
        const double cx = (t % nTX) * TILE + (s + 0.5) * (TILE / SPB) - 0.5 * W;
        const double cy = (t / nTX) * TILE_H + 0.5 * TILE_H - 0.5 * H;
        d[g] = {cx * cx + cy * cy, g};
    }
    std::stable_sort(d.begin(), d.end());
    for (int g = 0; g < n; ++g) order[g] = d[g].second;
}

int raster_order_len(int H, int W) { return raster_tiles(H, W, nullptr) * SPB; }

int raster_tiles(int H, int W, int* nTX) {
    const int tx = (W + TILE - 1) / TILE, ty = (H + TILE_H - 1) / TILE_H;
    if (nTX) *nTX = tx;
    return tx * ty;
}

// Candidates per grid chunk: as many as keep CHUNK_BYTES of splat records + cull
// bounds (80 B per splat) in flight, a multiple of 8 (the XCD count).
#ifndef GGS_CHUNK_MB
#define GGS_CHUNK_MB 40
#endif
constexpr int64_t CHUNK_BYTES = (int64_t)GGS_CHUNK_MB << 20;
int raster_chunk(int N) {
    const int64_t per = (int64_t)(N > 1 ? N : 1) * (int64_t)(sizeof(SplatRec) + sizeof(int4));
    int64_t ch = CHUNK_BYTES / per;
    if (ch > (1 << 24)) ch = 1 << 24;
    ch &= ~int64_t(7);
    return ch < 8 ? 8 : (int)ch;
}

// SIMDs (CUs x 4) of HIP device `dev`, for the single-round block order; 0 if
// unknown (no reordering).  Callers pass their context's device
// (DevCtx::simds), not the current one.
int device_simds(int dev) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return 4 * cus;
}

hipError_t launch_raster(hipStream_t st, int mode, const SplatRec* recs, const int4* bnds, int B, int N, int H, int W,
                         const float bg[3], float* img, const float4* plan, float* partials,
                         const int* tile_order, const unsigned char* dirty, const float* clean,
                         const int* live, const FinFused* fin, int simds) {
    int nTX;
    const int nTiles = raster_tiles(H, W, &nTX);
    const dim3 grid((unsigned)((int64_t)B * nTiles * SPB)), block(NT);
    const bool sat = N > SAT_MIN_SPLATS;
    const dim3 block_f(GGS_DEPTH_SPLIT && !sat ? 2 * NT : NT);   // fitness instances (depth split: 2 waves)
    const int CH = raster_chunk(N);
    const FinFused ff = (mode != 0 && fin) ? *fin : FinFused{};
    if (GGS_DEPTH_SPLIT) simds = 0;
    // FUSED is a template parameter, so the instances without the fold carry none
    // of its code (a runtime test left the SA raster 1 % slower than round 3's)
#define GGS_RASTER(M, S, F)                                                                    \
    hipLaunchKernelGGL((raster_kernel<M, S, F>), grid, (M) ? block_f : block, 0, st, recs, bnds, B, N, H, W, nTX, nTiles, \
                       bg[0], bg[1], bg[2], img, plan, partials, tile_order, dirty, clean, live, CH, ff, simds)
    // the saturation check only where strip lists can grow long (N > SAT_MIN_SPLATS);
    // at the bench's 256 splats the kernel without it is the faster code (+1.6 %)
    if (mode == 0) { if (!sat) GGS_RASTER(0, false, false); else GGS_RASTER(0, true, false); }   // image
    else if (!ff.ctr) { if (!sat) GGS_RASTER(1, false, false); else GGS_RASTER(1, true, false); }   // fitness
    else { if (!sat) GGS_RASTER(1, false, true); else GGS_RASTER(1, true, true); }  // + folded finalize
#undef GGS_RASTER
    return hipGetLastError();
}

hipError_t launch_finalize(hipStream_t st, const float* partials, const float* wpartials, int B,
                           int nTiles, int mode, int H, int W, float* out, const int* live) {
    // 4 strip partials per (candidate, tile)
    hipLaunchKernelGGL(finalize_kernel, dim3((B + 3) / 4), dim3(256), 0, st, partials, wpartials, nTiles * 4,
                       mode, (double)H * (double)W, B, out, live);
    return hipGetLastError();
}

}  // namespace ggs

#if GGS_TIMING
extern "C" int ggs_debug_timing_read(void* host, size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(ggs::g_ggs_timing), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
#endif
