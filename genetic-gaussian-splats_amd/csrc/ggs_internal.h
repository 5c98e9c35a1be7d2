// Internal declarations shared by ggs_kernels.hip and ggs_capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ggs.h"

// Diagnostic knobs (per-wave clocks, a plan-less traffic probe that computes the
// wrong fitness, saturation / cull / chunk overrides) compile only into the probe
// library (`make probe` -> libggs_probe.so, which ggs/_lib.py refuses unless
// GGS_PROBE=1), never into libggs.so.
#if !defined(GGS_PROBE_BUILD) &&                                                         \
    (defined(GGS_NOPLAN) || defined(GGS_TIMING) || defined(GGS_VTIMING) || defined(GGS_SATURATE) || \
     defined(GGS_SAT_EVERY) || defined(GGS_SAT_BATCH) || defined(GGS_SAT_AHEAD) ||             \
     defined(GGS_CULL_AHEAD) || defined(GGS_CHUNK_MB) || defined(GGS_NO_RATIO_CLAMP) ||               \
     defined(GGS_DEPTH_SPLIT) || defined(GGS_TILE_H))
#error "GGS_* diagnostic knobs are for the probe build only: make probe PROBE=\"-D...\""
#endif
#ifdef GGS_PROBE_BUILD
#define GGS_BUILD_KIND "probe"
#else
#define GGS_BUILD_KIND "product"
#endif

namespace ggs {

// One preprocessed splat as the raster kernel consumes it (64 B, HBM + LDS).
// cx, cy: centre in pixels (render.py:15-16); A, Bc, Cc, la: exp2-domain
// coefficients of the Gaussian (render.py:189-192 folded with log2(a));
// r, g, b: colour in [0,1] (render.py:40-42); x0..y1: inclusive integer AABB
// (render.py:27-30).
struct __attribute__((aligned(16))) SplatRec {
    // C64, r, g, b and rho sit in EVEN dwords: a 16-dword s_load lands them in
    // even SGPRs, the low half of an aligned SGPR pair, which the raster's v_pk_*
    // ops broadcast to both halves (op_sel_hi) with no per-visit copy (round 3:
    // raster -2.8 % vs odd dwords, which the compiler copied into even SGPRs).
    // (A, B8) is one aligned pair: one v_pk_mul forms (A qx, 8 Bc qx) per visit.
    // The raster works with qy / 8 (cy8): C64 = 64 Cc, B8 = 8 Bc and c128 = 128 Cc
    // are the exponent's y-terms rescaled by powers of two (exact), so the
    // recurrence ratio needs no separate 8 * bx (see make_rec).
    float C64, cx, r, cy8;
    float g, la, b, c128;
    float rho, rho4, A, B8;    // row-recurrence constants: 2^(128 Cc), 2^(64 Cc) (8-row step)
    int x0, x1, y0, y1;
};
static_assert(sizeof(SplatRec) == 64, "SplatRec must be 64 bytes");

// live (device, may be null): only the first *live candidates of N splats each are
// live (the device SA loop sizes its grids for the session's capacity and sets the
// round's neighbour count on the device); the other threads / waves exit at once.
// recs [S] and bnds [S] (the records' AABBs, compact for the raster's cull) go together.
hipError_t launch_prep(hipStream_t st, bool encode, const float* genomes, int64_t S, int C, int H,
                       int W, float k, SplatRec* recs, int4* bnds, float* f9, int* i4, float* enc9,
                       const int* live = nullptr, int n_per = 0);
int raster_tiles(int H, int W, int* nTX);
// The fitness finalize folded into the raster (MODE 1): each strip wave counts
// itself in ctr[b] after storing its partial, and the candidate's last strip
// wave reduces the candidate's partials (finalize_wave, so the same bits as
// finalize_kernel) into out[b] and resets ctr[b] to 0 for the next launch.
// ctr: one int per candidate of the launch, all zero before the first launch
// (ensure_zeroed); the counters are per workspace, so launches that may run at
// the same time (other streams) never share them.
struct FinFused {
    int* ctr = nullptr;               // null: no fusion (launch_finalize follows)
    const float* wpartials = nullptr;  // the plan's weight block
    float* out = nullptr;             // [B] fitness scalars
    double hw = 0.0;                  // H * W
    int mode = 0;                     // GGS_FIT_*
};
// simds: SIMDs of the launch's device (DevCtx::simds; 0 = unknown: no single-round
// reordering).
hipError_t launch_raster(hipStream_t st, int mode, const SplatRec* recs, const int4* bnds, int B, int N, int H, int W,
                         const float bg[3], float* img, const float4* plan, float* partials,
                         const int* tile_order, const unsigned char* dirty = nullptr,
                         const float* clean = nullptr, const int* live = nullptr, const FinFused* fin = nullptr,
                         int simds = 0);
// SIMDs (CUs x 4) of HIP device `dev`, 0 if unknown.
int device_simds(int dev);

// Strips touched by splats that differ between the neighbours and the current
// state (old AABB from cur_recs, new from nb_recs) -> dirty [n][tiles][4] (zeroed
// first).  rule 1: a splat differs when its raster record does (nb_recs [n][N] vs
// cur_recs [N]); rule 0: when its genes do (nb [n][N][9] vs curr [N][9]).
hipError_t launch_dirty(hipStream_t st, const float* curr, const float* nb, const SplatRec* cur_recs,
                        const SplatRec* nb_recs, int n, int N, int H, int W, unsigned char* dirty,
                        unsigned* n_changed, const int* live = nullptr, int rule = 1);
// Target plan for the fitness epilogue (built once per target/mask/mode/beta).
// wblock (plan_wsum_bytes): the plan's Sum w as a double, then per-wave sums.
hipError_t launch_plan(hipStream_t st, const float* target, const float* mask, int mode, float beta,
                       int H, int W, float4* plan, float* wblock);
size_t plan_bytes(int H, int W);
size_t plan_wsum_bytes(int H, int W);
// Tile visiting order for the raster grid: tiles sorted by distance of their
// centre from the image centre (central tiles carry the most splats; running
// them first shortens the tail of the launch).
void raster_tile_order(int H, int W, int* order);   // raster_order_len(H, W) entries
int raster_order_len(int H, int W);
hipError_t launch_detmath(hipStream_t st, const float* x, const float* y, int64_t n, int fn,
                          float* out);
hipError_t launch_finalize(hipStream_t st, const float* partials, const float* wpartials, int B,
                           int nTiles, int mode, int H, int W, float* out, const int* live = nullptr);

// ---- device GA (ggs_ga.hip) -------------------------------------------------
struct GaParamsDev {            // one generation's operator parameters (float32 as the host path)
    float sig_xy, sig_alog, sig_blog, sig_theta, sig_rgb, sig_alpha;   // build_mut_sigma
    float mutpb, cxpb;
    int tour_k;
    int mutate_only;            // SA neighbours: every offspring = mutation of pop[0], no selection
    int o_base;                 // Philox key offset of offspring 0 (SA: index of the first try)
    float log_lo, log_hi;       // clamp_genome scale bounds (utils.py:38-39)
};
struct GaDrawsDev {             // explicit draws (device pointers); all NULL -> Philox in-kernel
    const int* tour_idx;        // [P*k]
    const int* perm;            // [P]
    const int* cx;              // [npairs]
    const float* cx_u;          // [npairs*N]
    const float *u_xy, *u_ab;   // [P*N*2]
    const float *u_t, *u_rgb, *u_a;   // [P*N]
    const int *k_color, *k_xy, *k_ab, *k_t;   // [P]
    const float *n_xy, *n_ab;   // [P*N*2]
    const float* n_t;           // [P*N]
    const float* n_rgba;        // [P*N*4]
    const int *swap_i, *swap_pick;    // [P]
    const double* swap_u;       // [P]
};
struct GaBestDev {
    double* fit;
    int* src;
    int* updated;
    float* ind;                 // [N*9]
};
// ---- device SA loop (ggs_sa_run) ---------------------------------------------
// Tries are numbered globally, g = it * tries + k.  A round mutates the next
// `live` tries from the current state (Philox keyed by (seed, it, k), as
// ggs_sa_propose), evaluates them, and the accept kernel walks them in order
// (annealing.py:133-150): the first acceptance installs that neighbour and ends
// the round (the later tries came from the old state and are re-proposed by the
// next round); without one the round consumes all `live` tries.
struct SaLoopDev {
    int64_t pos, end;           // next try / one past the chunk's last try
    int32_t live;               // neighbours of the current round (0: chunk done)
    int32_t acc_j;              // neighbour the last round accepted (-1: none)
    int32_t new_best;           // ... and whether it became the best
    int32_t tries, first_it;    // tries per iteration; iteration of sit[0]
    int32_t cap, width;         // neighbour capacity; fixed width (0: adaptive)
    int32_t pad_;
    double acc_rate;            // EWMA of acceptances per try (ggs/annealing.py)
    double best_fit;
    double curr_fit;            // float32 energy of the current state, widened
    uint64_t evaluated, rounds, accepted;
    double width_r;             // adaptive width: a round's fixed cost / its cost per neighbour
};
// Adaptive round width: the w in [1, cap] with the least expected cost per consumed
// try.  A round of w neighbours costs ~ (r + w) neighbour-evaluations and consumes
// E(w) = (1 - (1 - p)^w) / p tries at acceptance rate p (it ends at the first
// acceptance); p -> 0: E = w, so w = cap.  Only the cost depends on w: the
// trajectory is the same at every width.
__host__ __device__ inline int sa_width_rule(double p, int cap, double r) {
    if (cap <= 1) return 1;
    if (!(p > 1e-9)) return cap;
    int best_w = 1;
    double best = 0.0, qw = 1.0;
    for (int w = 1; w <= cap; ++w) {
        qw *= 1.0 - p;
        const double cost = (r + w) * p / (1.0 - qw);
        if (w == 1 || cost < best) { best = cost; best_w = w; }
    }
    return best_w;
}
struct SaItDev {                // one iteration of the chunk
    float sig[6];               // build_mut_sigma at this iteration
    float pad_[2];
    double T;                   // temperature (annealing.py:29-44)
};
// The end of a device round (one workgroup): the neighbours' fitness from their
// strip partials (finalize_wave), the acceptance walk, the install of the
// accepted neighbour (genome; records and strip partials too when cur_recs is
// set, for the incremental path), curves[(it - first_it)*2 + {0,1}] = best,
// current after each iteration, and the next round's mask-group flags.
struct SaRoundDev {
    const float* partials;      // [cap][nslots] the round's strip partials
    const float* wpartials;     // [nslots] plan weight sums
    int nslots, mode, N;
    double hw;
    float* fits_out;            // [cap] the round's energies (kept for inspection)
    uint64_t seed;
    float mutpb;
    double* curves;
    float *curr, *best;         // [N][9] state
    const float* nb;            // [cap][N][9] the round's neighbours
    SplatRec* cur_recs;         // incremental only (else null)
    const SplatRec* nb_recs;
    float* cur_part;
    int gcap;                   // the next round's neighbour limit: the batch's launch width
};
hipError_t launch_sa_accept(hipStream_t st, SaLoopDev* sl, const SaItDev* sit, const SaRoundDev& r);
// Start a chunk: pos/end/tries/first_it and the first round's width (at most gcap).
hipError_t launch_sa_begin(hipStream_t st, SaLoopDev* sl, int64_t pos, int64_t end, int tries, int first_it,
                           int cap, int width, double width_r, int gcap);
// Mask-group flags of the chunk's n_tries tries from pos0 (state-independent):
// tflags [n_tries], zeroed here.
hipError_t launch_sa_flags(hipStream_t st, int64_t pos0, int n_tries, int tries, uint64_t seed, float mutpb, int N,
                           int* tflags);
// The round's neighbours (Philox draws; the bits of ga_variation_kernel's
// mutate-only mode) with their raster records: tflags of the chunk's tries,
// sizes [cap][N] scratch, off [cap][N][9], recs [cap][N].
hipError_t launch_sa_mutate(hipStream_t st, const SaLoopDev* sl, const SaItDev* sit, const GaParamsDev& prm,
                            uint64_t seed, int N, int cap, const int* tflags, const float* curr, float* off,
                            float* sizes, SplatRec* recs, int4* bnds, int H, int W, float k_sigma);
// The acceptance uniform of try (it, k): Philox4x32-10 keyed by seed, 53-bit double
// in [0, 1).  Host and device compute the same bits.
double sa_accept_uniform(uint64_t seed, uint32_t it, uint32_t k);

struct BreedDev {               // the fused breed (launch_ga_variation with br != null)
    const float* pop_prev;      // [P][N][9] population P_{g-1} (materialised)
    const float* fits_prev;     // [P] its fitness
    const float* off_prev;      // [P][N][9] offspring of generation g-1
    const float* off_fits;      // [P] their fitness (finalize / all-gather)
    const int* elite_prev;      // [E] rows of P_{g-1} by rank (survivors / the previous breed)
    int* elite_next;            // [E] the same for P_g (written by the stats workgroup)
    float* pop_next;            // [P][N][9] P_g, row o written by workgroup o
    float* fits_next;           // [P]
    double* curves_row;         // [3] best, mean, median of P_g
    GaBestDev best;
    int elite_k;
};
hipError_t launch_ga_variation(hipStream_t st, const float* pop, const float* fits, int P, int N,
                               const GaParamsDev& prm, const GaDrawsDev& d, uint64_t seed, int gen,
                               float* off, int n_off,    // n_off offspring (GA: P; SA: tries)
                               SplatRec* recs = nullptr, int4* bnds = nullptr, int H = 0, int W = 0,
                               float k_sigma = 3.0f,
                               const SaLoopDev* sl = nullptr, const SaItDev* sit = nullptr,
                               const BreedDev* br = nullptr);
                               // recs != null: also prep the offspring (records [n_off][N]);
                               // sl != null: SA loop round (neighbour o = try sl->pos + o, its
                               // iteration's sigmas from sit; o >= sl->live exits)
struct FitReduce {               // survivors reduces the offspring's strip partials itself
    const float* partials = nullptr; // [P][nT] (null: use off_fits)
    const float* wpartials = nullptr;
    int nT = 0, mode = 0;
    double hw = 0.0;
};
hipError_t launch_ga_survivors(hipStream_t st, const float* fits, const float* off_fits, int P,
                               int elite_k, int* src, float* new_fits, const GaBestDev& best,
                               double* curves_row, int init, const FitReduce& fr = FitReduce{},
                               int* elite_next = nullptr);   // P <= 512: rows of the output by rank, rank < E
hipError_t launch_ga_gather(hipStream_t st, const float* pop, const float* off, int P, int N,
                            const int* src, float* next, const GaBestDev& best, int init);
int ga_max_population();
int ga_breed_max_population();   // the fused breed's population limit

// ---- RCCL (ggs_comm.cpp) ----------------------------------------------------
// Grouped in-place all-gather over single-process communicators (ggs_comm_init_local):
// buf[d] holds shard d at buf[d] + d*per; afterwards every buf[d] holds all n shards.
int comm_group_allgather_inplace(void* const* comms, int n, hipStream_t const* streams, float* const* bufs,
                                 int64_t per);

}  // namespace ggs
