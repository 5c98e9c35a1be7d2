// Device-resident genetic algorithm around the fitness pipeline (SURVEY.md §8f
// next #1: algorithm.py:85-141, genetic.py:8-91, utils.py:10-45 on the GPU).
//
// Per generation (all on one stream, no host round trip):
//   variation  1 workgroup / offspring: tournament (genetic.py:8-14), uniform
//              row crossover (:17-21), masked Gaussian mutation with the >=1-flag
//              guarantees (:32-77), wrap/clamp (utils.py:35-45), size-ordered
//              splat swap (:79-91).  Same float32 operation order as ggs/ga.py,
//              which is replay-verified against the reference.
//   fitness    prep + raster + finalize (ggs_kernels.hip) on the offspring
//   survivors  1 workgroup: stable sort of the parents' fitness -> elites,
//              next population = elites + offspring[:P-E] (algorithm.py:129-141),
//              best-so-far (:144-150) and the curves (:153-155)
//   gather     1 workgroup / individual: builds the next population buffer
// Draws come either from explicit per-generation arrays (replay / parity with the
// host path) or from a counter-based Philox4x32-10 generator keyed by
// (seed, generation, individual, splat), which needs no state between launches.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ggs_internal.h"
#include "ggs_prep.h"

namespace ggs {

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11), counter-based
// ---------------------------------------------------------------------------
struct U4 {
    uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = {(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

__device__ __forceinline__ float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }

// stream ids: which draw a 4-word Philox block feeds
enum : uint32_t { S_MASK = 1, S_NORM_A = 2, S_NORM_B = 3, S_NORM_C = 4, S_IND = 5, S_TOUR = 6, S_CX = 7,
                  S_ACCEPT = 8 };

// SA acceptance uniform of try (it, k): 53 bits of one Philox block -> [0, 1)
// (the role of random.random() at annealing.py:140-142).  Host and device.
__host__ __device__ __forceinline__ double accept_u(uint64_t seed, uint32_t it, uint32_t k) {
    const U4 r = philox({it, k, 0u, S_ACCEPT}, (uint32_t)seed, (uint32_t)(seed >> 32));
    return ((double)(r.x >> 5) * 67108864.0 + (double)(r.y >> 6)) * (1.0 / 9007199254740992.0);
}
double sa_accept_uniform(uint64_t seed, uint32_t it, uint32_t k) { return accept_u(seed, it, k); }

struct Rng {
    uint32_t k0, k1, gen;
    __device__ U4 block(uint32_t stream, uint32_t who, uint32_t what) const {
        return philox({gen, who, what, stream}, k0, k1);
    }
};

// Box-Muller pair from two Philox words: r = sqrt(-2 ln u1) with u1 in (0, 1],
// angle 2*pi*u2.  The hardware transcendentals (v_log_f32 = log2, v_sqrt_f32,
// v_sin/v_cos_f32 in revolutions) are ample for mutation noise and keep the
// per-splat draw chain short; both outputs are used (5 pairs cover a splat's 9).
__device__ __forceinline__ float2 normal_pair(uint32_t a, uint32_t b) {
    const float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);      // (0, 1]
    const float u2 = u01(b);                                               // [0, 1) revolutions
    const float r = __builtin_amdgcn_sqrtf(-1.38629436112f * __builtin_amdgcn_logf(u1));   // -2 ln 2 * log2
    return make_float2(r * __builtin_amdgcn_cosf(u2), r * __builtin_amdgcn_sinf(u2));
}

// ---------------------------------------------------------------------------
// float32 helpers with ggs/ga.py's exact semantics
// ---------------------------------------------------------------------------
constexpr float PI32 = 3.14159274101257324219f;     // float32(pi)
constexpr float TWO_PI32 = 6.28318548202514648438f; // float32(2*pi)

__device__ __forceinline__ float wrap_angle(float th) {      // np.remainder(th + pi, 2pi) - pi
    const float x = th + PI32;
    float r = fmodf(x, TWO_PI32);
    if (r != 0.0f && (r < 0.0f) != (TWO_PI32 < 0.0f)) r += TWO_PI32;
    return r - PI32;
}
__device__ __forceinline__ float clip(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// ---------------------------------------------------------------------------
// variation
// ---------------------------------------------------------------------------
__device__ int tournament_pick(const float* __restrict__ fits, const GaDrawsDev& d, const Rng& rng,
                               int q, int P, int k) {
    int best = -1;
    for (int j = 0; j < k; ++j) {
        int i;
        if (d.tour_idx) {
            i = d.tour_idx[q * k + j];
        } else {
            const U4 r = rng.block(S_TOUR, (uint32_t)q, (uint32_t)j);
            i = min((int)(u01(r.x) * (float)P), P - 1);
        }
        if (best < 0 || fits[i] < fits[best]) best = i;        // genetic.py:11-13: strict <
    }
    return best;
}

// Per-splat pieces of the variation, shared by the GA variation kernel and the
// SA loop's split kernels (same code, so the same bits).
struct MaskU {                  // mask uniforms of one splat (genetic.py:37-54)
    float ux0, ux1, ua0, ua1, ut, urgb, ua;
};
__device__ __forceinline__ MaskU mask_draws(const GaDrawsDev& d, const Rng& rng, uint32_t og, int64_t ob, int s) {
    MaskU m;
    if (d.u_xy) {
        m.ux0 = d.u_xy[(ob + s) * 2]; m.ux1 = d.u_xy[(ob + s) * 2 + 1];
        m.ua0 = d.u_ab[(ob + s) * 2]; m.ua1 = d.u_ab[(ob + s) * 2 + 1];
        m.ut = d.u_t[ob + s]; m.urgb = d.u_rgb[ob + s]; m.ua = d.u_a[ob + s];
    } else {
        const U4 r1 = rng.block(S_MASK, og, (uint32_t)(2 * s));
        const U4 r2 = rng.block(S_MASK, og, (uint32_t)(2 * s + 1));
        m.ux0 = u01(r1.x); m.ux1 = u01(r1.y); m.ua0 = u01(r1.z); m.ua1 = u01(r1.w);
        m.ut = u01(r2.x); m.urgb = u01(r2.y); m.ua = u01(r2.z);
    }
    return m;
}
enum : int { ANY_COLOR = 1, ANY_XY = 2, ANY_AB = 4, ANY_T = 8 };
__device__ __forceinline__ int mask_any(const MaskU& m, float p) {
    return (((m.urgb < p) | (m.ua < p)) ? ANY_COLOR : 0) | (((m.ux0 < p) | (m.ux1 < p)) ? ANY_XY : 0) |
           (((m.ua0 < p) | (m.ua1 < p)) ? ANY_AB : 0) | ((m.ut < p) ? ANY_T : 0);
}
struct Fallback {               // genetic.py:24-29: one-true flat indices (-1: not needed)
    int kc, kx, kb, kt;
};
__device__ __forceinline__ Fallback fallbacks(const GaDrawsDev& d, const Rng& rng, uint32_t og, int o, int N,
                                              int any) {
    Fallback f{-1, -1, -1, -1};
    if (!(any & ANY_COLOR)) f.kc = d.k_color ? d.k_color[o] : (int)(rng.block(S_IND, og, 0).x % (uint32_t)(2 * N));
    if (!(any & ANY_XY)) f.kx = d.k_xy ? d.k_xy[o] : (int)(rng.block(S_IND, og, 1).x % (uint32_t)(2 * N));
    if (!(any & ANY_AB)) f.kb = d.k_ab ? d.k_ab[o] : (int)(rng.block(S_IND, og, 2).x % (uint32_t)(2 * N));
    if (!(any & ANY_T)) f.kt = d.k_t ? d.k_t[o] : (int)(rng.block(S_IND, og, 3).x % (uint32_t)N);
    return f;
}
struct NormD {                  // normals of one splat (genetic.py:57-70)
    float nx0, nx1, na0, na1, nt, nr0, nr1, nr2, nr3;
};
__device__ __forceinline__ NormD normal_draws(const GaDrawsDev& d, const Rng& rng, uint32_t og, int64_t ob, int s,
                                              int N) {
    NormD n;
    if (d.u_xy) {
        n.nx0 = d.n_xy[(ob + s) * 2]; n.nx1 = d.n_xy[(ob + s) * 2 + 1];
        n.na0 = d.n_ab[(ob + s) * 2]; n.na1 = d.n_ab[(ob + s) * 2 + 1];
        n.nt = d.n_t[ob + s];
        n.nr0 = d.n_rgba[(ob + s) * 4]; n.nr1 = d.n_rgba[(ob + s) * 4 + 1];
        n.nr2 = d.n_rgba[(ob + s) * 4 + 2]; n.nr3 = d.n_rgba[(ob + s) * 4 + 3];
    } else {
        const U4 g1 = rng.block(S_NORM_A, og, (uint32_t)s);
        const U4 g2 = rng.block(S_NORM_B, og, (uint32_t)s);
        const U4 g3 = rng.block(S_NORM_C, og, (uint32_t)s);
        const float2 p1 = normal_pair(g1.x, g1.y), p2 = normal_pair(g1.z, g1.w);
        const float2 p3 = normal_pair(g2.x, g2.y), p4 = normal_pair(g2.z, g2.w);
        const float2 p5 = normal_pair(g3.x, g3.y);
        n.nx0 = p1.x; n.nx1 = p1.y; n.na0 = p2.x; n.na1 = p2.y;
        n.nt = p3.x; n.nr0 = p3.y; n.nr1 = p4.x; n.nr2 = p4.y; n.nr3 = p5.x;
    }
    return n;
}
// genetic.py:37-70 + clamp_genome (utils.py:35-45) on one row, ggs/ga.py's float32 op order
__device__ __forceinline__ void mutate_row(float* g, const MaskU& u, const NormD& n, const Fallback& f, int s,
                                           const GaParamsDev& prm) {
    const float p = prm.mutpb;
    const bool mrgb = (u.urgb < p) || (f.kc == 2 * s), ma = (u.ua < p) || (f.kc == 2 * s + 1);
    const bool mx0 = (u.ux0 < p) || (f.kx == 2 * s), mx1 = (u.ux1 < p) || (f.kx == 2 * s + 1);
    const bool mb0 = (u.ua0 < p) || (f.kb == 2 * s), mb1 = (u.ua1 < p) || (f.kb == 2 * s + 1);
    const bool mt = (u.ut < p) || (f.kt == s);
    g[0] = g[0] + (n.nx0 * prm.sig_xy) * (float)mx0;
    g[1] = g[1] + (n.nx1 * prm.sig_xy) * (float)mx1;
    g[2] = g[2] + (n.na0 * prm.sig_alog) * (float)mb0;
    g[3] = g[3] + (n.na1 * prm.sig_blog) * (float)mb1;
    g[4] = g[4] + (n.nt * prm.sig_theta) * (float)mt;
    g[4] = wrap_angle(g[4]);
    g[5] = g[5] + (n.nr0 * prm.sig_rgb) * (float)mrgb;
    g[6] = g[6] + (n.nr1 * prm.sig_rgb) * (float)mrgb;
    g[7] = g[7] + (n.nr2 * prm.sig_rgb) * (float)mrgb;
    g[8] = g[8] + (n.nr3 * prm.sig_alpha) * (float)ma;
    g[0] = clip(g[0], 0.0f, 1.0f);
    g[1] = clip(g[1], 0.0f, 1.0f);
    g[2] = clip(g[2], prm.log_lo, prm.log_hi);
    g[3] = clip(g[3], prm.log_lo, prm.log_hi);
    g[4] = wrap_angle(g[4]);
#pragma unroll
    for (int c = 5; c < 9; ++c) g[c] = clip(g[c], 0.0f, 255.0f);
}

// ---------------------------------------------------------------------------
// breed: survivors + gather of the previous generation fused into the variation
// ---------------------------------------------------------------------------
constexpr int ST = 1024;   // max threads; the launch uses min(ST, pow2 >= P) (cheap barriers at P=128)
constexpr int SMAX = 4096;
constexpr int RANKMAX = 512;   // counting ranks below this population size (and the fused breed's limit)

// Every breed workgroup rebuilds, in LDS, the next population P_g of
// algorithm.py:129-141 as a row map: row r < E is the parent of rank r (stable
// order of the parents' fitness: elite_prev, written by whoever produced that
// fitness vector — the survivors kernel or the previous breed's stats
// workgroup, from the same counting rank), row r >= E is offspring r - E of the
// generation just evaluated.  s_src[r] follows the survivors kernel's index
// space (parents 0..P-1, offspring P + q), s_nf[r] is the row's fitness.  The
// rows themselves are read from where they are (no gather in front of the
// tournament).
__device__ __forceinline__ int breed_src(const BreedDev& br, int r, int P, int E) {
    return r < E ? br.elite_prev[r] : P + (r - E);
}
__device__ __forceinline__ float breed_fit(const BreedDev& br, int src, int P) {
    return src < P ? br.fits_prev[src] : br.off_fits[src - P];
}
__device__ void breed_rows(const BreedDev& br, int P, float* s_nf, int* s_src) {
    const int E = br.elite_k < 1 ? 1 : br.elite_k;                      // algorithm.py:129
    for (int r = threadIdx.x; r < P; r += blockDim.x) {
        const int src = breed_src(br, r, P, E);
        s_src[r] = src;
        s_nf[r] = breed_fit(br, src, P);
    }
    __syncthreads();
}
__device__ __forceinline__ const float* breed_row(const BreedDev& br, int src, int P, int N) {
    return src < P ? br.pop_prev + (int64_t)src * N * 9 : br.off_prev + (int64_t)(src - P) * N * 9;
}
// The breed grid's extra workgroup: best so far (algorithm.py:143-150), the curves
// row (:153-155; sequential float64 mean, statistics.median), the best row — the
// survivors kernel's arithmetic on the same row map, so the same bits — and the
// next breed's elite list (the median's ranks, rank < E).
__device__ void breed_stats(const BreedDev& br, int P, int N, const float* s_nf, const int* s_src) {
    __shared__ float med[2];
    __shared__ int s_g, s_upd;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int E = br.elite_k < 1 ? 1 : br.elite_k;
    if (tid == 0) {
        int g = 0;
        double sum = (double)s_nf[0];
        for (int r = 1; r < P; ++r) {
            if (s_nf[r] < s_nf[g]) g = r;
            sum += (double)s_nf[r];
        }
        const double fg = (double)s_nf[g];
        const int upd = fg + 1e-10 < *br.best.fit;
        if (upd) {
            *br.best.fit = fg;
            *br.best.src = s_src[g];
        }
        *br.best.updated = upd;
        br.curves_row[0] = *br.best.fit;
        br.curves_row[1] = sum / (double)P;
        s_g = g;
        s_upd = upd;
    }
    for (int r = tid; r < P; r += nt) {
        const float f = s_nf[r];
        int rank = 0;
        for (int j = 0; j < P; ++j) rank += (s_nf[j] < f) | ((s_nf[j] == f) & (j < r));
        if (rank == P / 2) med[1] = f;
        if (rank == P / 2 - 1) med[0] = f;
        if (rank < E) br.elite_next[rank] = r;
    }
    __syncthreads();
    if (tid == 0) br.curves_row[2] = (P & 1) ? (double)med[1] : ((double)med[0] + (double)med[1]) / 2.0;
    if (s_upd) {
        const float* from = breed_row(br, s_src[s_g], P, N);
        for (int64_t i = tid; i < (int64_t)N * 9; i += nt) br.best.ind[i] = from[i];
    }
}

#ifndef GGS_VTIMING
#define GGS_VTIMING 0             // diagnostic build: per-workgroup phase clocks (tools/probe/breed_timing.py)
#endif
#if GGS_VTIMING
__device__ unsigned long long g_ggs_vtiming[8 * 4096];
#define GGS_VMARK(k) do { if (threadIdx.x == 0 && blockIdx.x < 4096) \
    g_ggs_vtiming[8 * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define GGS_VMARK(k) do { } while (0)
#endif

// Threads per variation workgroup (one workgroup per offspring): the smallest of
// 256 / 512 / 1024 that gives every splat its own thread up to 1,024 splats (the
// register-resident path below); 256 past that, and 1024 when a few large
// offspring are bred (SA tries at configs[4]: 4,096 splats each), which otherwise
// leave 16 splats per thread on a handful of CUs.  Results do not depend on VT
// (per-splat work, an OR, a sum and an in-order search).
//
// BREED: the generation's survivors and gather run inside this kernel (one extra
// workgroup, o == n_off, keeps best and curves): the parents are the rows of the
// next population P_g (breed_rows), each workgroup o also writes row o of P_g
// (and its fitness) for the generation after.  pop / fits are unused then.
template <int VT, bool BREED>
__global__ void __launch_bounds__(VT)
ga_variation_kernel(const float* __restrict__ pop, const float* __restrict__ fits, int P, int N,
                    GaParamsDev prm, GaDrawsDev d, uint32_t k0, uint32_t k1, int gen,
                    float* __restrict__ off, int n_off, SplatRec* __restrict__ recs, int4* __restrict__ bnds,
                    int H, int W, float k_sigma,
                    const SaLoopDev* __restrict__ sl, const SaItDev* __restrict__ sit, BreedDev br) {
    __shared__ int s_a, s_b, s_cx, s_any;
    __shared__ float s_nf[BREED ? RANKMAX : 1];
    __shared__ int s_src[BREED ? RANKMAX : 1];
    __shared__ float s_sizei;
    __shared__ int s_j, s_count;
    __shared__ int s_scan[VT / 64];
    const int o = blockIdx.x;                  // offspring index
    GGS_VMARK(0);
    const int pair = o >> 1;
    const bool first = (o & 1) == 0;
    const int tid = threadIdx.x;

    uint32_t og = (uint32_t)(o + prm.o_base);   // Philox identity of this offspring
    if (sl) {   // SA loop round: neighbour o is global try pos + o = (it, k); it's sigmas from sit
        if (o >= sl->live) return;
        const int64_t g = sl->pos + o;
        const int it = (int)(g / sl->tries);
        og = (uint32_t)(g % sl->tries);
        gen = it;
        const SaItDev& q = sit[it - sl->first_it];
        prm.sig_xy = q.sig[0]; prm.sig_alog = q.sig[1]; prm.sig_blog = q.sig[2];
        prm.sig_theta = q.sig[3]; prm.sig_rgb = q.sig[4]; prm.sig_alpha = q.sig[5];
    }
    if (BREED && o == n_off) {                 // the stats workgroup
        breed_rows(br, P, s_nf, s_src);
        breed_stats(br, P, N, s_nf, s_src);
        return;
    }
    const Rng rng{k0, k1, (uint32_t)gen};
    float* __restrict__ O = off + (int64_t)o * N * 9;
    const float p = prm.mutpb;
    const int64_t ob = (int64_t)o * N;
    const int E = br.elite_k < 1 ? 1 : br.elite_k;

    if (N <= VT) {
        // One splat per thread (s = tid).  Phase A issues everything that does not
        // depend on the parents' fitness — the row-map and gather loads (BREED),
        // the tournament's candidate indices, the crossover decision, every
        // per-splat draw — with no barrier in between, so the loads' latency
        // hides behind the Philox / Box-Muller arithmetic; after one barrier
        // thread 0 only compares fitness values.  The row, its draws and its size
        // then stay in registers / LDS from mutation to swap to prep.  Same
        // operations on the same values as the generic path, so the same bits.
        constexpr int KT = 32;                 // tournament picks precomputed when 2k <= 2*KT
        __shared__ int s_tour[2 * KT];
        __shared__ float s_size[VT];
        __shared__ float s_rowi[9], s_rowj[9];
        const int sp = tid;
        const bool act = sp < N;
        const int k = prm.tour_k;
        const bool pre = !prm.mutate_only && 2 * k <= 2 * KT;
        // --- phase A
        int msrc[(RANKMAX + VT - 1) / VT];               // BREED: row map entries r = tid + VT*i
        float mfit[(RANKMAX + VT - 1) / VT];
        float cp[9];                           // BREED: this thread's part of row o of P_g
        if (BREED) {
#pragma unroll
            for (int i = 0; i < (RANKMAX + VT - 1) / VT; ++i) {
                const int r = tid + VT * i;
                msrc[i] = r < P ? breed_src(br, r, P, E) : 0;
                mfit[i] = r < P ? breed_fit(br, msrc[i], P) : 0.0f;
            }
            const float* __restrict__ from = breed_row(br, breed_src(br, o, P, E), P, N);
#pragma unroll
            for (int c = 0; c < 9; ++c) {
                const int i = tid + VT * c;
                cp[c] = i < N * 9 ? from[i] : 0.0f;
            }
        }
        if (tid == 0) {
            s_any = 0;
            s_j = -1;
            if (prm.mutate_only) {
                s_a = 0;                       // annealing.py:122-128: mutate the current state
                s_b = 0;
                s_cx = 0;
            } else {
                s_cx = d.cx ? d.cx[pair] : (u01(rng.block(S_CX, (uint32_t)pair, 0).x) < prm.cxpb);
            }
        }
        if (pre && tid < 2 * k) {              // candidate j of parent h's tournament (genetic.py:11)
            const int h = tid / k, j = tid % k;
            const int q = h == 0 ? (d.perm ? d.perm[2 * pair] : 2 * pair)
                                 : (d.perm ? d.perm[(2 * pair + 1) % P] : (2 * pair + 1) % P);
            s_tour[tid] = d.tour_idx ? d.tour_idx[q * k + j]
                                     : min((int)(u01(rng.block(S_TOUR, (uint32_t)q, (uint32_t)j).x) * (float)P), P - 1);
        }
        MaskU u{};
        NormD nd{};
        float cxu = 0.0f;
        int any = 0;
        if (act) {
            u = mask_draws(d, rng, og, ob, sp);
            any = mask_any(u, p);
            if (!prm.mutate_only)
                cxu = d.cx_u ? d.cx_u[(int64_t)pair * N + sp]
                             : u01(rng.block(S_CX, (uint32_t)pair, (uint32_t)(sp + 1)).x);   // shared by the pair
            nd = normal_draws(d, rng, og, ob, sp, N);
        }
        if (BREED) {
#pragma unroll
            for (int i = 0; i < (RANKMAX + VT - 1) / VT; ++i) {
                const int r = tid + VT * i;
                if (r < P) {
                    s_src[r] = msrc[i];
                    s_nf[r] = mfit[i];
                }
            }
            fits = s_nf;
        }
        __syncthreads();
        GGS_VMARK(1);
        // --- tournament (genetic.py:8-14, strict <) on the fitness now in place;
        //     the mask groups' any() (genetic.py:24-29) meanwhile
        if (tid == 0 && !prm.mutate_only) {
            if (pre) {
                int best = -1;
                for (int j = 0; j < k; ++j) {
                    const int i = s_tour[j];
                    if (best < 0 || fits[i] < fits[best]) best = i;
                }
                s_a = best;
                best = -1;
                for (int j = 0; j < k; ++j) {
                    const int i = s_tour[k + j];
                    if (best < 0 || fits[i] < fits[best]) best = i;
                }
                s_b = best;
            } else {
                const int qa = d.perm ? d.perm[2 * pair] : 2 * pair;
                const int qb = d.perm ? d.perm[(2 * pair + 1) % P] : (2 * pair + 1) % P;
                s_a = tournament_pick(fits, d, rng, qa, P, k);
                s_b = tournament_pick(fits, d, rng, qb, P, k);
            }
        }
        {
            const int wa = (__ballot(any & ANY_COLOR) ? ANY_COLOR : 0) | (__ballot(any & ANY_XY) ? ANY_XY : 0) |
                           (__ballot(any & ANY_AB) ? ANY_AB : 0) | (__ballot(any & ANY_T) ? ANY_T : 0);
            if ((tid & 63) == 0 && wa) atomicOr(&s_any, wa);
        }
        __syncthreads();
        GGS_VMARK(2);
        any = s_any;
        const Fallback fb = fallbacks(d, rng, og, o, N, any);
        const float* __restrict__ A = BREED ? breed_row(br, s_src[s_a], P, N) : pop + (int64_t)s_a * N * 9;
        const float* __restrict__ Bp = BREED ? breed_row(br, s_src[s_b], P, N) : pop + (int64_t)s_b * N * 9;
        GGS_VMARK(3);
        float g[9];
        if (act) {
            // genetic.py:17-21 (c1 = where(m, a, b), c2 = where(m, b, a)) / duplicate
            const bool m = cxu < 0.5f;
            const bool takeA = s_cx ? (first ? m : !m) : first;
            const float* src = (takeA ? A : Bp) + (int64_t)sp * 9;
#pragma unroll
            for (int c = 0; c < 9; ++c) g[c] = src[c];
            mutate_row(g, u, nd, fb, sp, prm);
            s_size[sp] = expf(g[2]) * expf(g[3]);
        }
        if (N >= 2) {
            // genetic.py:79-91: pick i, then the pick-th later splat bigger than i
            const int i = d.swap_i ? d.swap_i[o] : (int)(rng.block(S_IND, og, 4).x % (uint32_t)(N - 1));
            __syncthreads();
            GGS_VMARK(4);
            const float sizei = s_size[i];
            const bool c = act && sp > i && s_size[sp] > sizei;
            const uint64_t bal = __ballot(c);
            const int lane = tid & 63, w = tid >> 6;
            if (lane == 0) s_scan[w] = __popcll(bal);
            __syncthreads();
            int count = 0, before = 0;
            for (int q = 0; q < VT / 64; ++q) {
                before += q < w ? s_scan[q] : 0;
                count += s_scan[q];
            }
            if (count > 0) {
                int pick;
                if (d.swap_pick && d.swap_pick[o] >= 0) pick = d.swap_pick[o];
                else {
                    const double uu = d.swap_u ? d.swap_u[o] : (double)u01(rng.block(S_IND, og, 5).x);
                    pick = (int)(uu * (double)count);
                    if (pick > count - 1) pick = count - 1;
                }
                const int inwave = __popcll(bal & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
                if (c && before + inwave == pick) s_j = sp;       // the (pick+1)-th in splat order
                __syncthreads();
                const int j = s_j;
                if (sp == i) {
#pragma unroll
                    for (int q = 0; q < 9; ++q) s_rowi[q] = g[q];
                }
                if (sp == j) {
#pragma unroll
                    for (int q = 0; q < 9; ++q) s_rowj[q] = g[q];
                }
                __syncthreads();
                if (sp == i) {
#pragma unroll
                    for (int q = 0; q < 9; ++q) g[q] = s_rowj[q];
                }
                if (sp == j) {
#pragma unroll
                    for (int q = 0; q < 9; ++q) g[q] = s_rowi[q];
                }
            }
        }
        GGS_VMARK(5);
        if (act) {
#pragma unroll
            for (int c = 0; c < 9; ++c) O[(int64_t)sp * 9 + c] = g[c];
            if (recs) {         // prep fused in (ggs_prep.h): the raster's record of this splat
                float row[9];
                encode_row(g, row);
                const SplatRec r = make_rec(preprocess_row(row, H, W, k_sigma));
                recs[ob + sp] = r;
                bnds[ob + sp] = rec_bounds(r);
            }
        }
        if (BREED) {            // gather: row o of P_g and its fitness, for the generation after
            float* __restrict__ to = br.pop_next + (int64_t)o * N * 9;
#pragma unroll
            for (int c = 0; c < 9; ++c) {
                const int i = tid + VT * c;
                if (i < N * 9) to[i] = cp[c];
            }
            if (tid == 0) br.fits_next[o] = s_nf[o];
        }
#if GGS_VTIMING
        __syncthreads();
#endif
        GGS_VMARK(6);
        return;
    }

    // ---- generic path (N > VT: several splats per thread) ------------------------
    if (BREED) {
        breed_rows(br, P, s_nf, s_src);
        const float* __restrict__ from = breed_row(br, s_src[o], P, N);     // gather: row o of P_g
        float* __restrict__ to = br.pop_next + (int64_t)o * N * 9;
        for (int64_t i = tid; i < (int64_t)N * 9; i += VT) to[i] = from[i];
        if (tid == 0) br.fits_next[o] = s_nf[o];
        fits = s_nf;
    }
    if (tid == 0 && prm.mutate_only) {
        s_a = 0;                               // annealing.py:122-128: mutate the current state
        s_b = 0;
        s_cx = 0;
    } else if (tid == 0) {
        // parents 2*pair and 2*pair+1 of the (shuffled) tournament winners
        const int qa = d.perm ? d.perm[2 * pair] : 2 * pair;
        const int qb = d.perm ? d.perm[(2 * pair + 1) % P] : (2 * pair + 1) % P;
        s_a = tournament_pick(fits, d, rng, qa, P, prm.tour_k);
        s_b = tournament_pick(fits, d, rng, qb, P, prm.tour_k);
        if (d.cx) s_cx = d.cx[pair];
        else s_cx = u01(rng.block(S_CX, (uint32_t)pair, 0).x) < prm.cxpb;
    }
    __syncthreads();
    const float* __restrict__ A = BREED ? breed_row(br, s_src[s_a], P, N) : pop + (int64_t)s_a * N * 9;
    const float* __restrict__ Bp = BREED ? breed_row(br, s_src[s_b], P, N) : pop + (int64_t)s_b * N * 9;

    // pass 1: crossover + mask flags, any() per mask group
    int any = 0;
    for (int s = tid; s < N; s += VT) any |= mask_any(mask_draws(d, rng, og, ob, s), p);
    any = (__syncthreads_or(any & ANY_COLOR) ? ANY_COLOR : 0) | (__syncthreads_or(any & ANY_XY) ? ANY_XY : 0) |
          (__syncthreads_or(any & ANY_AB) ? ANY_AB : 0) | (__syncthreads_or(any & ANY_T) ? ANY_T : 0);
    // genetic.py:24-29: fallback flat indices (k into [N,2] or [N,1] row-major)
    const Fallback fb = fallbacks(d, rng, og, o, N, any);

    // pass 2: build the child row, mutate, wrap, clamp -> off
    for (int s = tid; s < N; s += VT) {
        const MaskU u = mask_draws(d, rng, og, ob, s);
        const NormD nd = normal_draws(d, rng, og, ob, s, N);
        float cxu = 0.0f;
        if (s_cx) cxu = d.cx_u ? d.cx_u[(int64_t)pair * N + s]
                               : u01(rng.block(S_CX, (uint32_t)pair, (uint32_t)(s + 1)).x);   // shared by the pair
        // genetic.py:17-21 (c1 = where(m, a, b), c2 = where(m, b, a)) / duplicate
        const bool m = cxu < 0.5f;
        const bool takeA = s_cx ? (first ? m : !m) : first;
        const float* src = (takeA ? A : Bp) + (int64_t)s * 9;
        float g[9];
#pragma unroll
        for (int c = 0; c < 9; ++c) g[c] = src[c];
        mutate_row(g, u, nd, fb, s, prm);      // flags with the one-true fallbacks, mutation, clamp
#pragma unroll
        for (int c = 0; c < 9; ++c) O[(int64_t)s * 9 + c] = g[c];
    }
    if (N >= 2) {
    __syncthreads();   // workgroup-scope ordering of the rows just written

    // genetic.py:79-91: pick i, then the pick-th later splat bigger than i
    int i;
    if (d.swap_i) i = d.swap_i[o];
    else i = (int)(rng.block(S_IND, og, 4).x % (uint32_t)(N - 1));
    if (tid == 0) {
        s_sizei = expf(O[(int64_t)i * 9 + 2]) * expf(O[(int64_t)i * 9 + 3]);
        s_j = -1;
    }
    __syncthreads();
    const float sizei = s_sizei;
    int cnt = 0;
    for (int s = tid; s < N; s += VT)
        cnt += (s > i) && (expf(O[(int64_t)s * 9 + 2]) * expf(O[(int64_t)s * 9 + 3]) > sizei);
    {   // total candidates: workgroup sum
        const int lane = tid & 63, w = tid >> 6;
        int v = cnt;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) s_scan[w] = v;
        __syncthreads();
        if (tid == 0) {
            int tot = 0;
            for (int k = 0; k < VT / 64; ++k) tot += s_scan[k];
            s_count = tot;
        }
        __syncthreads();
    }
    const int count = s_count;
    if (count > 0) {
    int pick;
    if (d.swap_pick && d.swap_pick[o] >= 0) pick = d.swap_pick[o];
    else {
        const double u = d.swap_u ? d.swap_u[o] : (double)u01(rng.block(S_IND, og, 5).x);
        pick = (int)(u * (double)count);
        if (pick > count - 1) pick = count - 1;
    }
    // find the (pick+1)-th candidate in splat order: walk 256-splat chunks
    int seen = 0;
    for (int base = 0; base < N; base += VT) {
        const int s = base + tid;
        const bool c = s < N && s > i &&
                       (expf(O[(int64_t)s * 9 + 2]) * expf(O[(int64_t)s * 9 + 3]) > sizei);
        // exclusive prefix of c across the workgroup (in s order)
        const uint64_t bal = __ballot(c);
        const int lane = tid & 63, w = tid >> 6;
        const int inwave = __popcll(bal & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
        __syncthreads();
        if (lane == 0) s_scan[w] = __popcll(bal);
        __syncthreads();
        int before = seen;
        for (int k = 0; k < w; ++k) before += s_scan[k];
        if (c && before + inwave == pick) s_j = s;
        int tot = 0;
        for (int k = 0; k < VT / 64; ++k) tot += s_scan[k];
        seen += tot;
        __syncthreads();
        if (s_j >= 0) break;
    }
    const int j = s_j;
    if (tid < 9 && j >= 0) {
        const float a = O[(int64_t)i * 9 + tid], b = O[(int64_t)j * 9 + tid];
        O[(int64_t)i * 9 + tid] = b;
        O[(int64_t)j * 9 + tid] = a;
    }
    }   // count > 0
    }   // N >= 2
    if (recs) {             // prep fused in (ggs_prep.h): the raster's records of this offspring
        __syncthreads();    // swapped rows visible to the workgroup
        for (int s = tid; s < N; s += VT) {
            float row[9];
            encode_row(O + (int64_t)s * 9, row);
            const SplatRec r = make_rec(preprocess_row(row, H, W, k_sigma));
            recs[(int64_t)o * N + s] = r;
            bnds[(int64_t)o * N + s] = rec_bounds(r);
        }
    }
}

// ---------------------------------------------------------------------------
// survivors: elites by stable fitness order, next fitness vector, best, curves
// ---------------------------------------------------------------------------

// bitonic sort of n2 (power of two) LDS keys (+ optional indices), ascending;
// ties by index: lexicographic (key, idx) == Python's stable sorted()
__device__ void bitonic(float* key, int* idx, int n2) {
    const int nt = blockDim.x;
    for (int k = 2; k <= n2; k <<= 1) {
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
            for (int i = threadIdx.x; i < n2; i += nt) {
                const int l = i ^ jj;
                if (l > i) {
                    const bool up = (i & k) == 0;
                    const bool gt = key[i] > key[l] || (idx && key[i] == key[l] && idx[i] > idx[l]);
                    if (gt == up) {
                        const float tk = key[i]; key[i] = key[l]; key[l] = tk;
                        if (idx) { const int ti = idx[i]; idx[i] = idx[l]; idx[l] = ti; }
                    }
                }
            }
            __syncthreads();
        }
    }
}

__global__ void __launch_bounds__(ST)
ga_survivors_kernel(const float* __restrict__ fits, const float* __restrict__ off_fits, int P,
                    int elite_k, int* __restrict__ src, float* __restrict__ new_fits,
                    GaBestDev best, double* __restrict__ curves_row, int init, FitReduce fr,
                    int* __restrict__ elite_next) {
    // The surviving offspring's fitness (rows E..P-1 of the next generation):
    // given, or reduced here from the raster's strip partials, one wave per
    // candidate (finalize_wave: the same bits as finalize_kernel).
    const int E0 = elite_k < 1 ? 1 : elite_k;
    __shared__ float nf[SMAX];           // the next generation's fitness vector
    if (!init && fr.partials) {          // one wave per candidate
        const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
        for (int q = wave; q < P - E0; q += nw) {
            const float f = finalize_wave(fr.partials, fr.wpartials, fr.nT, fr.mode, fr.hw, q);
            if ((threadIdx.x & 63) == 0) {
                nf[E0 + q] = f;
                new_fits[E0 + q] = f;
                src[E0 + q] = P + q;                                // offspring q
            }
        }
    } else if (!init) {                  // one thread per candidate
        for (int q = threadIdx.x; q < P - E0; q += blockDim.x) {
            const float f = off_fits[q];
            nf[E0 + q] = f;
            new_fits[E0 + q] = f;
            src[E0 + q] = P + q;
        }
    }
    __shared__ float key[SMAX];
    __shared__ int idx[SMAX];
    const int tid = threadIdx.x, nt = blockDim.x;
    const int E = elite_k < 1 ? 1 : elite_k;                      // algorithm.py:129
    if (P <= RANKMAX) {
        // Small populations: ranks by counting (one LDS pass per element, 3
        // barriers) instead of two bitonic sorts (~60 barriers).  rank(r) = #{j:
        // (f_j, j) < (f_r, r)} is the position in Python's stable sorted().
        __shared__ float med[2];
        for (int r = tid; r < P; r += nt) key[r] = fits[r];
        __syncthreads();
        if (!init) {
            for (int r = tid; r < P; r += nt) {
                const float f = key[r];
                int rank = 0;
                for (int j = 0; j < P; ++j) rank += (key[j] < f) | ((key[j] == f) & (j < r));
                if (rank < E) {                                   // an elite, from the parents
                    src[rank] = r;
                    new_fits[rank] = f;
                    nf[rank] = f;
                }
            }
            // rows E..P-1 (the offspring) were written above
        } else {
            for (int r = tid; r < P; r += nt) nf[r] = key[r];
        }
        __syncthreads();
        if (tid == 0) {
            int g = 0;
            double sum = (double)nf[0];                           // sum(fitnesses) / len, in order
            for (int r = 1; r < P; ++r) {
                if (nf[r] < nf[g]) g = r;
                sum += (double)nf[r];
            }
            const double fg = (double)nf[g];
            if (init || fg + 1e-10 < *best.fit) {
                *best.fit = fg;
                *best.src = init ? g : src[g];
                *best.updated = 1;
            } else {
                *best.updated = 0;
            }
            curves_row[0] = *best.fit;
            curves_row[1] = sum / (double)P;
        }
        for (int r = tid; r < P; r += nt) {                       // statistics.median
            const float f = nf[r];
            int rank = 0;
            for (int j = 0; j < P; ++j) rank += (nf[j] < f) | ((nf[j] == f) & (j < r));
            if (rank == P / 2) med[1] = f;
            if (rank == P / 2 - 1) med[0] = f;
            if (elite_next && rank < E) elite_next[rank] = r;    // the fused breed's row map
        }
        __syncthreads();
        if (tid == 0)
            curves_row[2] = (P & 1) ? (double)med[1] : ((double)med[0] + (double)med[1]) / 2.0;
        return;
    }
    int n2 = 1;
    while (n2 < P) n2 <<= 1;
    if (!init) {
        for (int i = tid; i < n2; i += nt) {
            key[i] = i < P ? fits[i] : __builtin_inff();
            idx[i] = i < P ? i : 0x7fffffff;
        }
        __syncthreads();
        bitonic(key, idx, n2);
        for (int r = tid; r < E; r += nt) {                       // the elites, from the parents
            src[r] = idx[r];
            new_fits[r] = key[r];
            nf[r] = key[r];
        }
    } else {
        for (int r = tid; r < P; r += nt) nf[r] = fits[r];
    }
    __syncthreads();
    // best so far (algorithm.py:64-67, 143-150) and curves (:71-75, 153-155)
    if (tid == 0) {
        int g = 0;
        double sum = (double)nf[0];                               // sum(fitnesses) / len, in order
        for (int r = 1; r < P; ++r) {
            if (nf[r] < nf[g]) g = r;
            sum += (double)nf[r];
        }
        const double fg = (double)nf[g];
        if (init || fg + 1e-10 < *best.fit) {
            *best.fit = fg;
            *best.src = init ? g : src[g];
            *best.updated = 1;
        } else {
            *best.updated = 0;
        }
        curves_row[0] = *best.fit;
        curves_row[1] = sum / (double)P;
    }
    // median: sort the new fitness values (statistics.median on the list)
    for (int i = tid; i < n2; i += nt) key[i] = i < P ? nf[i] : __builtin_inff();
    __syncthreads();
    bitonic(key, nullptr, n2);
    if (tid == 0)
        curves_row[2] = (P & 1) ? (double)key[P / 2] : ((double)key[P / 2 - 1] + (double)key[P / 2]) / 2.0;
}

// next population rows from (parents | offspring) by src; best row if improved
__global__ void __launch_bounds__(256)
ga_gather_kernel(const float* __restrict__ pop, const float* __restrict__ off, int P, int N,
                 const int* __restrict__ src, float* __restrict__ next, GaBestDev best, int init) {
    const int r = blockIdx.x;
    const int sidx = init ? r : src[r];
    const float* from = sidx < P ? pop + (int64_t)sidx * N * 9 : off + (int64_t)(sidx - P) * N * 9;
    float* to = next + (int64_t)r * N * 9;
    const int64_t n = (int64_t)N * 9;
    if (!init)
        for (int64_t i = threadIdx.x; i < n; i += 256) to[i] = from[i];
    if (*best.updated && *best.src == sidx)      // the new best individual
        for (int64_t i = threadIdx.x; i < n; i += 256) best.ind[i] = from[i];
}

// ---------------------------------------------------------------------------
hipError_t launch_ga_variation(hipStream_t st, const float* pop, const float* fits, int P, int N,
                               const GaParamsDev& prm, const GaDrawsDev& d, uint64_t seed, int gen,
                               float* off, int n_off, SplatRec* recs, int4* bnds, int H, int W, float k_sigma,
                               const SaLoopDev* sl, const SaItDev* sit, const BreedDev* br) {
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    // The smallest workgroup that holds one splat per thread (the register-resident
    // path, N <= VT) up to 1,024 splats: the shipped GA run (config.py: 512 splats)
    // on the generic path (two splats per thread, the child rows round-tripping
    // through HBM between the passes) bred in 21.6 us per generation.
    // Past 1,024 splats (the generic path, several splats per thread) 256 threads,
    // unless the launch is too small to fill the chip (< 64 workgroups): the same
    // rule for the breed (+ stats workgroup) and the plain variation launch.
    const int vt = N <= 256 ? 256 : N <= 512 ? 512 : (N <= 1024 || n_off < 64) ? 1024 : 256;
#define GGS_VAR(VTT, BR, NB, BD)                                                                  \
    hipLaunchKernelGGL((ga_variation_kernel<VTT, BR>), dim3(NB), dim3(VTT), 0, st, pop, fits, P, N, prm, d, k0, \
                       k1, gen, off, n_off, recs, bnds, H, W, k_sigma, sl, sit, BD)
    if (br) {       // + the stats workgroup
        if (P > RANKMAX || n_off != P) return hipErrorInvalidValue;
        if (vt == 256) GGS_VAR(256, true, n_off + 1, *br);
        else if (vt == 512) GGS_VAR(512, true, n_off + 1, *br);
        else GGS_VAR(1024, true, n_off + 1, *br);
    } else {
        if (vt == 256) GGS_VAR(256, false, n_off, BreedDev{});
        else if (vt == 512) GGS_VAR(512, false, n_off, BreedDev{});
        else GGS_VAR(1024, false, n_off, BreedDev{});
    }
#undef GGS_VAR
    return hipGetLastError();
}

hipError_t launch_ga_survivors(hipStream_t st, const float* fits, const float* off_fits, int P,
                               int elite_k, int* src, float* new_fits, const GaBestDev& best,
                               double* curves_row, int init, const FitReduce& fr, int* elite_next) {
    int nt = fr.partials ? 512 : 64;   // 8 waves for the fused per-candidate reductions
    while (nt < P && nt < ST) nt <<= 1;
    hipLaunchKernelGGL(ga_survivors_kernel, dim3(1), dim3(nt), 0, st, fits, off_fits, P, elite_k,
                       src, new_fits, best, curves_row, init, fr, elite_next);
    return hipGetLastError();
}

hipError_t launch_ga_gather(hipStream_t st, const float* pop, const float* off, int P, int N,
                            const int* src, float* next, const GaBestDev& best, int init) {
    hipLaunchKernelGGL(ga_gather_kernel, dim3(P), dim3(256), 0, st, pop, off, P, N, src, next, best,
                       init);
    return hipGetLastError();
}

int ga_max_population() { return SMAX; }
#if GGS_VTIMING
extern "C" int ggs_debug_vtiming_read(void* host, size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ggs_vtiming), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
#endif
int ga_breed_max_population() { return RANKMAX; }

// ---------------------------------------------------------------------------
// device SA loop (ggs_sa_run): chunk start, and one round's acceptance walk
// ---------------------------------------------------------------------------
// Round width: the host loop's rule (ggs/annealing.py) without its iteration
// boundary — 1/acceptance rate, or the capacity while acceptances are rarer than that.
// gcap: the width of the batch of rounds the host enqueued (their launch width,
// <= cap): the host applies sa_width_rule at each sync, so every launched
// neighbour slot is used (an unused slot's early-exit strip waves are not free)
__device__ __forceinline__ int sa_width(const SaLoopDev& s, int gcap) {
    int w = gcap > 0 ? gcap : s.width;
    if (w <= 0) w = sa_width_rule(s.acc_rate, s.cap, s.width_r);
    w = min(w, s.cap);
    return (int)min((int64_t)w, max(s.end - s.pos, (int64_t)0));
}

// The round's neighbours, spread over the GPU: ga_variation_kernel gives each
// neighbour one workgroup, so a round of a few 4,096-splat neighbours ran on a
// few CUs (40 us + a 5-us prep launch).  Here three kernels of one workgroup per
// (neighbour, 256 splats) — flags, mutate + prep, swap — do the same per-splat
// work with the same helpers (the same bits as ggs_sa_propose's variation).
constexpr int SA_VT = 256;

struct SaTry {                  // neighbour o of the round -> its Philox identity and sigmas
    uint32_t og;
    int gen;
};
__device__ __forceinline__ SaTry sa_try(const SaLoopDev& s, const SaItDev* sit, int o, GaParamsDev& prm) {
    const int64_t g = s.pos + o;
    const int it = (int)(g / s.tries);
    const SaItDev& q = sit[it - s.first_it];
    prm.sig_xy = q.sig[0]; prm.sig_alog = q.sig[1]; prm.sig_blog = q.sig[2];
    prm.sig_theta = q.sig[3]; prm.sig_rgb = q.sig[4]; prm.sig_alpha = q.sig[5];
    return {(uint32_t)(g % s.tries), it};
}

// pass 1, for every try of the chunk at once (the mask uniforms do not depend on
// the state, so a try re-proposed after an acceptance keeps its flags): any() of
// each mask group over try t's splats -> tflags[t] (OR; zeroed by the caller)
__global__ void __launch_bounds__(SA_VT)
sa_flags_kernel(int64_t pos0, int tries, uint32_t k0, uint32_t k1, float mutpb, int N, int nch,
                int* __restrict__ tflags) {
    const int t = blockIdx.x / nch, s = (blockIdx.x % nch) * SA_VT + threadIdx.x;
    const int64_t g = pos0 + t;
    const Rng rng{k0, k1, (uint32_t)(g / tries)};
    const int any = s < N ? mask_any(mask_draws(GaDrawsDev{}, rng, (uint32_t)(g % tries), 0, s), mutpb) : 0;
    const int wave_any = (__ballot(any & ANY_COLOR) ? ANY_COLOR : 0) | (__ballot(any & ANY_XY) ? ANY_XY : 0) |
                         (__ballot(any & ANY_AB) ? ANY_AB : 0) | (__ballot(any & ANY_T) ? ANY_T : 0);
    if ((threadIdx.x & 63) == 0 && wave_any) atomicOr(&tflags[t], wave_any);
}

hipError_t launch_sa_flags(hipStream_t st, int64_t pos0, int n_tries, int tries, uint64_t seed, float mutpb, int N,
                           int* tflags) {
    const int nch = (N + SA_VT - 1) / SA_VT;
    hipError_t e = hipMemsetAsync(tflags, 0, sizeof(int) * (size_t)n_tries, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sa_flags_kernel, dim3((unsigned)((int64_t)n_tries * nch)), dim3(SA_VT), 0, st, pos0, tries,
                       (uint32_t)seed, (uint32_t)(seed >> 32), mutpb, N, nch, tflags);
    return hipGetLastError();
}

// pass 2: mutate each splat of the current state into neighbour o, its raster
// record, and its size exp(a)exp(b) for the swap
__global__ void __launch_bounds__(SA_VT)
sa_mutate_kernel(const SaLoopDev* __restrict__ sl, const SaItDev* __restrict__ sit, GaParamsDev prm, uint32_t k0,
                 uint32_t k1, int N, int nch, const int* __restrict__ tflags, const float* __restrict__ curr,
                 float* __restrict__ off, float* __restrict__ sizes, SplatRec* __restrict__ recs,
                 int4* __restrict__ bnds, int H, int W, float k_sigma) {
    const int o = blockIdx.x / nch, s = (blockIdx.x % nch) * SA_VT + threadIdx.x;
    if (o >= sl->live || s >= N) return;
    const SaTry t = sa_try(*sl, sit, o, prm);
    const Rng rng{k0, k1, (uint32_t)t.gen};
    const GaDrawsDev d{};
    const SaLoopDev& sv = *sl;
    const Fallback fb = fallbacks(d, rng, t.og, o, N, tflags[sv.pos + o - (int64_t)sv.first_it * sv.tries]);
    const MaskU u = mask_draws(d, rng, t.og, 0, s);
    const NormD nd = normal_draws(d, rng, t.og, 0, s, N);
    float g[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) g[c] = curr[(int64_t)s * 9 + c];
    mutate_row(g, u, nd, fb, s, prm);
    const int64_t os = (int64_t)o * N + s;
#pragma unroll
    for (int c = 0; c < 9; ++c) off[os * 9 + c] = g[c];
    sizes[os] = expf(g[2]) * expf(g[3]);
    float row[9];
    encode_row(g, row);
    const SplatRec r = make_rec(preprocess_row(row, H, W, k_sigma));
    recs[os] = r;
    bnds[os] = rec_bounds(r);
}

// genetic.py:79-91 on neighbour o: the pick-th later splat bigger than a random
// splat i trades rows (and raster records) with it.  Thread t owns the contiguous
// run of splats [t*per, (t+1)*per) (splat order = thread order), counts its
// candidates in one read of the sizes, one workgroup scan of the counts gives the
// total (-> pick) and each run's rank offset, and the thread whose run holds the
// pick walks its run again to name j.  Two barriers (the first version counted,
// then walked the sizes in 1024-splat chunks with three barriers per chunk: 8.4 us
// per round at 4,096 splats).
constexpr int SW_THREADS = 1024;
__global__ void __launch_bounds__(SW_THREADS)
sa_swap_kernel(const SaLoopDev* __restrict__ sl, uint32_t k0, uint32_t k1, int N, const float* __restrict__ sizes,
               float* __restrict__ off, SplatRec* __restrict__ recs, int4* __restrict__ bnds) {
    __shared__ int s_wsum[SW_THREADS / 64], s_j;
    const int o = blockIdx.x, tid = threadIdx.x;
    const SaLoopDev& sv = *sl;
    if (o >= sv.live || N < 2) return;
    const int64_t g = sv.pos + o;
    const uint32_t og = (uint32_t)(g % sv.tries);
    const Rng rng{k0, k1, (uint32_t)(g / sv.tries)};
    const float* __restrict__ sz = sizes + (int64_t)o * N;
    const int i = (int)(rng.block(S_IND, og, 4).x % (uint32_t)(N - 1));
    const float sizei = sz[i];
    const int lane = tid & 63, w = tid >> 6;
    const int per = (N + SW_THREADS - 1) / SW_THREADS;
    const int r0 = min(tid * per, N), r1 = min(r0 + per, N);
    int cnt = 0;
    for (int sk = max(r0, i + 1); sk < r1; ++sk) cnt += sz[sk] > sizei;
    int v = cnt;                                       // inclusive wave scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(v, d);
        if (lane >= d) v += u;
    }
    if (lane == 63) s_wsum[w] = v;
    if (tid == 0) s_j = -1;
    __syncthreads();
    int before = v - cnt, count = 0;
#pragma unroll
    for (int q = 0; q < SW_THREADS / 64; ++q) {
        const int t = s_wsum[q];
        before += q < w ? t : 0;
        count += t;
    }
    if (count == 0) return;                            // (uniform)
    int pick = (int)((double)u01(rng.block(S_IND, og, 5).x) * (double)count);
    if (pick > count - 1) pick = count - 1;
    if (pick >= before && pick < before + cnt) {       // this run holds the (pick+1)-th candidate
        int left = pick - before;
        for (int sk = max(r0, i + 1); sk < r1; ++sk)
            if (sz[sk] > sizei && left-- == 0) {
                s_j = sk;
                break;
            }
    }
    __syncthreads();
    const int j = s_j;
    float* __restrict__ O = off + (int64_t)o * N * 9;
    if (tid < 9) {
        const float a = O[(int64_t)i * 9 + tid], b = O[(int64_t)j * 9 + tid];
        O[(int64_t)i * 9 + tid] = b;
        O[(int64_t)j * 9 + tid] = a;
    } else if (tid >= 64 && tid < 64 + 4) {           // a record is a function of its row alone
        float4* ri = reinterpret_cast<float4*>(recs + (int64_t)o * N + i) + (tid - 64);
        float4* rj = reinterpret_cast<float4*>(recs + (int64_t)o * N + j) + (tid - 64);
        const float4 a = *ri, b = *rj;
        *ri = b;
        *rj = a;
    } else if (tid == 128) {
        int4* bi = bnds + (int64_t)o * N + i;
        int4* bj = bnds + (int64_t)o * N + j;
        const int4 a = *bi, b = *bj;
        *bi = b;
        *bj = a;
    }
}

hipError_t launch_sa_mutate(hipStream_t st, const SaLoopDev* sl, const SaItDev* sit, const GaParamsDev& prm,
                            uint64_t seed, int N, int cap, const int* tflags, const float* curr, float* off,
                            float* sizes, SplatRec* recs, int4* bnds, int H, int W, float k_sigma) {
    const int nch = (N + SA_VT - 1) / SA_VT;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    hipLaunchKernelGGL(sa_mutate_kernel, dim3(cap * nch), dim3(SA_VT), 0, st, sl, sit, prm, k0, k1, N, nch, tflags,
                       curr, off, sizes, recs, bnds, H, W, k_sigma);
    hipLaunchKernelGGL(sa_swap_kernel, dim3(cap), dim3(SW_THREADS), 0, st, sl, k0, k1, N, sizes, off, recs, bnds);
    return hipGetLastError();
}

__global__ void sa_begin_kernel(SaLoopDev* sl, int64_t pos, int64_t end, int tries, int first_it, int cap,
                                int width, double width_r, int gcap) {
    SaLoopDev s = *sl;
    s.pos = pos;
    s.end = end;
    s.tries = tries;
    s.first_it = first_it;
    s.cap = cap;
    s.width = width;
    s.width_r = width_r;
    s.acc_j = -1;
    s.new_best = 0;
    s.live = sa_width(s, gcap);
    *sl = s;
}

// The end of a round, one workgroup: the neighbours' fitness (finalize_wave, the
// bits of finalize_kernel), then annealing.py:130-150 over them in try order by
// one thread, then the workgroup installs the accepted neighbour.  Same arithmetic as the
// host loop (ggs/annealing.py): dE in float64 from the float32 energies, the
// Metropolis test u < exp(-dE/T) (device exp; the host's math.exp agrees to the
// last ulp in all but rare cases, and u would have to fall between the two),
// the 1e-12 best margin.
__global__ void __launch_bounds__(1024)
sa_accept_kernel(SaLoopDev* __restrict__ sl, const SaItDev* __restrict__ sit, SaRoundDev r) {
    __shared__ int s_j, s_nb;
    __shared__ float fits[SMAX];
    const int N = r.N;
    {
        const int live = sl->live, nw = blockDim.x >> 6;
        for (int b = threadIdx.x >> 6; b < live; b += nw) {
            const float v = finalize_wave(r.partials, r.wpartials, r.nslots, r.mode, r.hw, b);
            if ((threadIdx.x & 63) == 0) {
                fits[b] = v;
                r.fits_out[b] = v;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t seed = r.seed;
        double* __restrict__ curves = r.curves;
        SaLoopDev s = *sl;
        int jacc = -1, nbest = 0;
        if (s.live > 0) {
            int used = s.live;
            for (int j = 0; j < s.live; ++j) {
                const int64_t g = s.pos + j;
                const int it = (int)(g / s.tries), k = (int)(g % s.tries);
                const double T = sit[it - s.first_it].T;
                const double e_new = (double)fits[j];
                const double dE = e_new - s.curr_fit;                       // annealing.py:133
                bool acc = dE <= 0.0;
                if (!acc && T > 0.0) acc = accept_u(seed, (uint32_t)it, (uint32_t)k) < exp(-dE / T);
                s.acc_rate = 0.9 * s.acc_rate + 0.1 * (acc ? 1.0 : 0.0);
                if (acc) s.curr_fit = e_new;
                const bool nbst = s.curr_fit + 1e-12 < s.best_fit;            // annealing.py:148-150
                if (nbst) s.best_fit = s.curr_fit;
                if (k == s.tries - 1) {                                     // end of iteration `it`
                    curves[2 * (int64_t)(it - s.first_it)] = s.best_fit;
                    curves[2 * (int64_t)(it - s.first_it) + 1] = s.curr_fit;
                }
                if (acc) {          // the later tries were mutated from the old state
                    jacc = j;
                    nbest = nbst;
                    used = j + 1;
                    s.accepted += 1;
                    break;
                }
            }
            s.evaluated += (uint64_t)s.live;
            s.rounds += 1;
            s.pos += used;
        }
        s.acc_j = jacc;
        s.new_best = nbest;
        s.live = sa_width(s, r.gcap);
        *sl = s;
        s_j = jacc;
        s_nb = nbest;
    }
    __syncthreads();
    const int j = s_j;
    if (j < 0) return;
    float* __restrict__ curr = r.curr;
    float* __restrict__ best = r.best;
    // install: 16-B copies (the genome is 36 N bytes: N % 4 floats of tail)
    const int64_t n9 = (int64_t)N * 9, n4 = n9 >> 2;
    const float* __restrict__ src = r.nb + j * n9;
    const float4* __restrict__ s4 = reinterpret_cast<const float4*>(src);
    float4* __restrict__ c4 = reinterpret_cast<float4*>(curr);
    float4* __restrict__ b4 = reinterpret_cast<float4*>(best);
    const bool nbst = s_nb;
    if (((j * n9) & 3) == 0) {
        // distinct buffers (restrict): the unrolled loads go out together instead of
        // one load-store round trip per iteration
#pragma unroll 8
        for (int64_t i = threadIdx.x; i < n4; i += blockDim.x) {
            const float4 v = s4[i];
            c4[i] = v;
            if (nbst) b4[i] = v;
        }
        for (int64_t i = 4 * n4 + threadIdx.x; i < n9; i += blockDim.x) {
            curr[i] = src[i];
            if (nbst) best[i] = src[i];
        }
    } else {
        for (int64_t i = threadIdx.x; i < n9; i += blockDim.x) {
            const float v = src[i];
            curr[i] = v;
            if (nbst) best[i] = v;
        }
    }
    if (r.cur_recs) {       // incremental evaluation keeps the state's records and partials
        const float4* rs = reinterpret_cast<const float4*>(r.nb_recs + j * (int64_t)N);
        float4* rd = reinterpret_cast<float4*>(r.cur_recs);
        for (int64_t i = threadIdx.x; i < 4 * (int64_t)N; i += blockDim.x) rd[i] = rs[i];
        for (int i = threadIdx.x; i < r.nslots; i += blockDim.x)
            r.cur_part[i] = r.partials[(int64_t)j * r.nslots + i];
    }
}

hipError_t launch_sa_begin(hipStream_t st, SaLoopDev* sl, int64_t pos, int64_t end, int tries, int first_it,
                           int cap, int width, double width_r, int gcap) {
    hipLaunchKernelGGL(sa_begin_kernel, dim3(1), dim3(1), 0, st, sl, pos, end, tries, first_it, cap, width,
                       width_r, gcap);
    return hipGetLastError();
}

hipError_t launch_sa_accept(hipStream_t st, SaLoopDev* sl, const SaItDev* sit, const SaRoundDev& r) {
    hipLaunchKernelGGL(sa_accept_kernel, dim3(1), dim3(1024), 0, st, sl, sit, r);
    return hipGetLastError();
}

}  // namespace ggs
