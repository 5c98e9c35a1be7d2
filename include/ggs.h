/*
 * ggs.h — C ABI of libggs.so, the MI355X (gfx950) 2D Gaussian-splat renderer and
 * fitness evaluator.  Plain pointers and sizes only; no torch/HIP types in any
 * signature (device streams are passed as void*).
 *
 * It is the drop-in boundary for the reference's hot path
 * (josedelrey/genetic-gaussian-splats):
 *
 *   ggs_render          <- modules/render.py:203-252  render_splats_rgb_triton
 *                          (with render.py:8-47 _preprocess_genome,
 *                           render.py:50-118 _gpu_bin_splats_to_tiles,
 *                           render.py:121-200 _render_tile_over_kernel)
 *   ggs_fitness         <- modules/fitness.py:7-31  fitness_many
 *                          (with modules/encode.py:62-79 genome_to_renderer_batched;
 *                           fitness.py:34-47 fitness_population is a host-side loop)
 *   ggs_encode          <- modules/encode.py:27-79  genome_to_renderer(_batched)
 *   ggs_preprocess      <- modules/render.py:8-47   _preprocess_genome
 *   ggs_*_device        the same two operations on caller-owned device memory
 *                        (inputs already resident in HBM, caller's HIP stream)
 *
 * Genome layouts (row-major float32, C >= 9 columns per splat, extra columns
 * ignored as render.py:222-223 does):
 *   axes-angle (fitness input, population.py:43):  x, y, a_log, b_log, theta, r, g, b, alpha
 *   renderer   (render input,  encode.py:37-57):   x, y, log l11, log l22, l21, r, g, b, alpha
 *
 * Ownership: all pointers are caller-owned and only used during the call (host
 * API: the call is synchronous; device API: the work is enqueued on `stream`
 * and the pointers must stay valid until it completes).  The library keeps
 * pooled device workspaces and a cache of the last target/mask uploaded per
 * device (keyed by size + a 64-bit content hash).
 *
 * Errors: 0 on success, a negative GGS_E* code otherwise; ggs_last_error()
 * returns a thread-local message.  The reference's assertion failures
 * (render.py:217 CUDA device, :219 ndim, :223 C >= 9) map to GGS_ENODEV and
 * GGS_EINVAL.  Thread safety: calls may come from any thread; each device
 * context is guarded by its own mutex.
 */
#ifndef GGS_H_
#define GGS_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GGS_OK 0
#define GGS_EINVAL (-1) /* bad argument (reference asserts render.py:219,223) */
#define GGS_ENODEV (-2) /* no usable HIP device (reference assert render.py:217) */
#define GGS_EHIP (-3)   /* HIP runtime / launch failure */
#define GGS_ENOMEM (-4) /* device or pinned host allocation failed */

/* fitness modes (fitness.py:17-31) */
#define GGS_FIT_NONE 0     /* weight_mask is None:  mean over H*W*3 of d^2          */
#define GGS_FIT_WEIGHTED 1 /* default GA path:      sum(w*d^2) / (sum(w) + 1e-12)   */
#define GGS_FIT_BOOST 2    /* boost_only=True:      mean(d^2*wb) / (mean(wb)+1e-12), wb = 1+beta*clamp(w,0,1) */

/* Library version string. */
const char* ggs_version(void);

/* Initialise up to max_devices HIP devices (<=0: all).  Returns the number of
 * usable devices (>0) or a negative error.  Idempotent; called lazily by every
 * entry point. */
int ggs_init(int32_t max_devices);

/* Number of HIP devices the library sees (0 before ggs_init / without GPUs). */
int ggs_device_count(void);

/* Restrict the host API's fan-out to the listed device ids, in order (n == 0:
 * all devices).  One process per GPU calls this with its local rank.  Device
 * contexts are created lazily on first use.  Returns the active count. */
int ggs_select_devices(const int32_t* ids, int32_t n);

/* Thread-local message describing the last error on this thread ("" if none). */
const char* ggs_last_error(void);

/* Free every device buffer, stream and pinned host buffer. */
void ggs_shutdown(void);

/* ---- host-pointer API (drop-in path) ----------------------------------------
 * render: genomes [B,N,C] renderer layout -> out [B,H,W,3] in [0,1].
 *   bg: background RGB (render.py:209, default 1,1,1); NULL means (1,1,1).
 * fitness: genomes [B,N,C] axes-angle layout, target [H,W,3], mask [H,W]
 *   (NULL iff mode == GGS_FIT_NONE) -> out [B] float32.
 * n_devices: shard the B candidates contiguously over the first n_devices of
 *   the active device list (<=0: all of them; see ggs_select_devices). */
int ggs_render(const float* genomes, int64_t B, int32_t N, int32_t C, int32_t H, int32_t W,
               float k_sigma, const float* bg, float* out_bhw3, int32_t n_devices);
int ggs_fitness(const float* genomes_axes, int64_t B, int32_t N, int32_t C, const float* target_hw3,
                const float* mask_hw, int32_t mode, float boost_beta, int32_t H, int32_t W,
                float k_sigma, float* out_B, int32_t n_devices);

/* ---- stage exports (host pointers; parity tests) ----------------------------
 * encode: S splat rows (stride C) axes-angle -> renderer rows [S,9].
 * preprocess: S renderer rows (stride C) -> out_f9 [9][S] = cx, cy, sxx, sxy,
 *   syy, rc, gc, bc, a and out_i4 [4][S] = x0, x1, y0, y1 (render.py:45-47). */
int ggs_encode(const float* genomes_axes, int64_t S, int32_t C, float* out_S9);
int ggs_preprocess(const float* genomes, int64_t S, int32_t C, int32_t H, int32_t W, float k_sigma,
                   float* out_f9, int32_t* out_i4);

/* Deterministic-math probe (parity tests of csrc/ggs_detmath.h against
 * oracle/detmath.py): out[i] = f(x[i]) for fn 0 exp, 1 log, 2 sin, 3 cos,
 * 4 sqrt (correctly rounded), 5 x[i] / y[i] (correctly rounded). */
int ggs_detmath_eval(int32_t fn, const float* x, const float* y, int64_t n, float* out);

/* ---- device-pointer API (inputs resident in HBM) ----------------------------
 * Same semantics as the host API on one device; all pointers are device
 * pointers on `device`; work is enqueued on `stream` (a hipStream_t, NULL =
 * the null stream) and the call returns without synchronising. */
int ggs_render_device(int32_t device, void* stream, const float* d_genomes, int64_t B, int32_t N,
                      int32_t C, int32_t H, int32_t W, float k_sigma, const float* bg,
                      float* d_out_bhw3);
int ggs_fitness_device(int32_t device, void* stream, const float* d_genomes_axes, int64_t B,
                       int32_t N, int32_t C, const float* d_target_hw3, const float* d_mask_hw,
                       int32_t mode, float boost_beta, int32_t H, int32_t W, float k_sigma,
                       float* d_out_B);

/* Target plan: the fitness epilogue's inputs (target, mask, mode, beta) laid out
 * once in the raster's lane order — what ggs_fitness_device rebuilds on every
 * call.  A caller whose target/mask stay fixed over a run (a GA loop) builds it
 * once (enqueued on `stream`; the inputs must stay valid until it has run) and
 * evaluates generations with ggs_fitness_device_planned (same results). */
int ggs_plan_create(int32_t device, void* stream, const float* d_target_hw3, const float* d_mask_hw,
                    int32_t mode, float boost_beta, int32_t H, int32_t W, void** plan);
int ggs_fitness_device_planned(void* plan, void* stream, const float* d_genomes_axes, int64_t B,
                               int32_t N, int32_t C, float k_sigma, float* d_out_B);
void ggs_plan_destroy(void* plan);

/* ---- device-resident GA ------------------------------
 * genetic_approx's generation loop (algorithm.py:85-155) on one device: the
 * population, fitness, elites, best individual and curves stay in HBM; a
 * generation is variation -> fitness -> survivors -> gather, no host sync.
 * Up to pop_size 512 the survivors/gather of a generation run inside the next
 * generation's variation launch ("breed"), and the fitness finalize inside the
 * raster launch (its last strip wave per candidate reduces): 2 launches per
 * generation instead of 5; ggs_ga_read applies the last generation's survivors
 * first, so what it returns is the same either way (GGS_GA_UNFUSED=1: separate
 * survivors/gather launches; GGS_UNFUSED_FINALIZE=1: a separate finalize launch).
 * Draws: explicit arrays (ggs_ga_step with draws != NULL; replay / parity) or a
 * counter-based Philox4x32-10 stream keyed by (seed, generation, individual). */
typedef struct ggs_ga_config {
    int32_t pop_size, n_splats, H, W, tour_k, elite_k;
    float cxpb, mutpb, k_sigma, min_scale_splats, max_scale_splats;
    float scale_log_lo, scale_log_hi; /* clamp bounds log(min), log(max*max(H,W)); 0,0 = compute */
    int32_t fitness_mode;             /* GGS_FIT_* */
    float boost_beta;
    int32_t schedule;                 /* 0 linear, 1 cosine, 2 exp (utils.py:14-27) */
    double sig_max[6], sig_min[6];    /* xy, alog, blog, theta, rgb, alpha (config.py:22-43) */
    uint64_t seed;
} ggs_ga_config;

typedef struct ggs_ga_draws {         /* host arrays for ONE generation (ggs/ga.py layout) */
    const int32_t* tour_idx;          /* [P*k]   random.randrange draws (genetic.py:11) */
    const int32_t* perm;              /* [P]     random.shuffle (algorithm.py:90) */
    const int32_t* cx;                /* [ceil(P/2)] crossover decisions (algorithm.py:97) */
    const float* cx_u;                /* [ceil(P/2)*N] crossover masks (genetic.py:18) */
    const float *u_xy, *u_ab;         /* [P*N*2] mask uniforms (genetic.py:37-38) */
    const float *u_t, *u_rgb, *u_a;   /* [P*N] */
    const int32_t *k_color, *k_xy, *k_ab, *k_t;   /* [P] one-true fallbacks (genetic.py:24-29) */
    const float *n_xy, *n_ab;         /* [P*N*2] normals (genetic.py:57-70) */
    const float* n_t;                 /* [P*N] */
    const float* n_rgba;              /* [P*N*4] */
    const int32_t *swap_i, *swap_pick;/* [P] swap draws (genetic.py:79-91); pick < 0 -> swap_u */
    const double* swap_u;             /* [P] */
} ggs_ga_draws;

/* init_pop [P,N,9] axes-angle (required); mask may be NULL iff fitness_mode is
 * GGS_FIT_NONE.  Evaluates the initial population. */
int ggs_ga_create(int32_t device, const ggs_ga_config* cfg, const float* target_hw3,
                  const float* mask_hw, const float* init_pop, void** handle);
/* Shard the device GA's fitness evaluation over the ranks of `comm` (one
 * process per GPU; every rank created its session with the same config, target,
 * mask, initial population and seed, and steps it with the same arguments —
 * checked: the ranks exchange a 64-bit fingerprint of those inputs and the call
 * fails with GGS_EINVAL on every rank if any differ):
 * each generation every rank breeds all P offspring (same draws), rasterises its
 * contiguous block of ceil(P/nranks), and one in-place RCCL all-gather of the
 * offspring fitness scalars lets every rank run the same survivors step, so the
 * populations stay identical without exchanging genomes (north_star: shard the
 * generation's candidates across the GPUs of a node).  comm = NULL: one GPU.
 * The communicator must outlive the session's use of it. */
int ggs_ga_set_comm(void* handle, void* comm);
int ggs_ga_step(void* handle, int32_t gen, int32_t total_gens, const ggs_ga_draws* draws);
int ggs_ga_run(void* handle, int32_t first_gen, int32_t n_gens, int32_t total_gens);
/* Synchronises; any output may be NULL.  curves: [n_curves][3] = best, mean, median. */
int ggs_ga_read(void* handle, float* pop, float* fits, float* best_ind, double* best_fit,
                double* curves, int32_t* n_curves);
void ggs_ga_destroy(void* handle);

/* ---- device-resident simulated-annealing neighbours (annealing.py:121-150) ---
 * The current state stays on the GPU.  ggs_sa_propose mutates it into n
 * neighbours — tries first_try .. first_try+n-1 of iteration `it`, draws either
 * explicit (ggs_ga_draws layout, mutation fields only, indexed by local try) or
 * Philox keyed by (seed, it, try), so a try's neighbour does not depend on how
 * the tries are batched — evaluates them in one launch and returns their
 * energies.  The host runs the acceptance test (annealing.py:133-146) and
 * ggs_sa_commit installs the accepted neighbour j (and/or snapshots the best).
 * cfg: pop_size = the largest n per propose call; tour_k/elite_k/cxpb unused.
 * Replaces: annealing.py:122-131 (duplicate + mutate_individual + fitness). */
int ggs_sa_create(int32_t device, const ggs_ga_config* cfg, const float* target_hw3,
                  const float* mask_hw, const float* init_ind, void** handle, float* init_fit);
int ggs_sa_propose(void* handle, int32_t it, int32_t total_iters, int32_t first_try, int32_t n,
                   const ggs_ga_draws* draws, float* fits_out);
/* j >= 0: current <- neighbour j of the last propose; update_best: best <- current. */
int ggs_sa_commit(void* handle, int32_t j, int32_t update_best);
/* Synchronises; any output may be NULL.  neighbours: [n of the last propose][N][9]. */
int ggs_sa_read(void* handle, float* current, float* best, float* neighbours);
/* The SA loop itself on the device (annealing.py:117-155 for iterations
 * first_it .. first_it+n_its-1): each round mutates the next tries from the
 * current state (Philox keyed by (seed, it, try), as ggs_sa_propose), evaluates
 * them in one launch and walks them in order with the Metropolis test of
 * annealing.py:133-146 — acceptance uniform ggs_sa_accept_uniform(seed, it, try)
 * — installing the first accepted neighbour (and the best, :148-150) on the GPU;
 * the host syncs once per batch of rounds, not per try.  temps[i]: temperature of
 * iteration first_it+i (annealing.py:29-44, the caller's float64); width:
 * neighbours per round, 0 = adaptive (1 / acceptance rate, at most pop_size);
 * results do not depend on it.  curves_out[i] = {best, current} energy after
 * iteration first_it+i (annealing.py:152-155).  A session is driven either by
 * ggs_sa_run or by ggs_sa_propose/commit, not both. */
int ggs_sa_run(void* handle, int32_t first_it, int32_t n_its, int32_t total_iters, int32_t tries,
               const double* temps, int32_t width, double* curves_out);
/* ggs_sa_run's batching rule (pure host arithmetic, no device): rounds enqueued
 * before the next host sync when `remaining` tries of the chunk are left and a
 * round is expected to consume `est` of them — ceil(remaining / est), at least
 * 1, at most GGS_SA_MAX_ROUNDS_PER_SYNC (a bound on the dispatches queued
 * between syncs: 4 per round, 6 with incremental evaluation). */
#define GGS_SA_MAX_ROUNDS_PER_SYNC 64
int64_t ggs_sa_rounds_per_sync(int64_t remaining, int32_t est);
/* The device loop's state after the last ggs_sa_run (any output may be NULL). */
int ggs_sa_loop_state(void* handle, double* best_fit, double* curr_fit, uint64_t* rounds,
                      uint64_t* evaluated, uint64_t* accepted);
/* The acceptance uniform in [0, 1) ggs_sa_run draws for try k of iteration it
 * (lets a host loop reproduce the device loop's trajectory). */
int ggs_sa_accept_uniform(uint64_t seed, int32_t it, int32_t k, double* u);
/* Incremental evaluation (default off): a neighbour's 16-column strips that no
 * changed splat touches (old or new AABB) keep the current state's partial sums —
 * bit-identical to a full re-render; off = every strip is rasterised.  Turning
 * it on re-evaluates the current state's records and strip partials (the device
 * loop keeps them only while it is on), so it may be toggled between calls. */
int ggs_sa_set_incremental(void* handle, int32_t on);
/* Neighbours proposed and splats found changed (summed over proposals). */
int ggs_sa_stats(void* handle, uint64_t* proposed, uint64_t* changed_splats);
void ggs_sa_destroy(void* handle);

/* ---- multi-GPU fitness gather -------------------------------
 * One process per GPU; candidates are sharded in contiguous blocks and the only
 * exchange is an all-gather of each rank's fitness scalars over RCCL (xGMI).
 * Replaces nothing in the reference (single-device, render.py:4); it is the
 * collective of the sharded fitness_population (fitness.py:34-47).  RCCL is
 * loaded at first use (the copy already in the process, else $GGS_RCCL, else the
 * one beside the HIP runtime, by absolute path) and must come from the HIP
 * runtime's directory.  Rank 0 makes the id, every rank passes the same bytes. */
#define GGS_COMM_ID_BYTES 128
int ggs_comm_unique_id(uint8_t* id128);
int ggs_comm_create(int32_t device, int32_t nranks, int32_t rank, const uint8_t* id128, void** comm);
/* recv[r*count + i] = rank r's send[i] (device pointers).  overlap = 0: enqueued
 * on `stream` after the work already there; *ticket = -1.  overlap = 1: runs on
 * the communicator's own stream once the work already on `stream` is done, and
 * `stream` continues at once; *ticket names it for ggs_comm_wait (the caller
 * must not overwrite d_send or read d_recv before waiting). */
int ggs_comm_allgather(void* comm, void* stream, const float* d_send, float* d_recv, int64_t count,
                       int32_t overlap, int64_t* ticket);
/* Make `stream` wait (on the device, no host sync) for the gather `ticket`;
 * valid for the 64 most recent tickets. */
int ggs_comm_wait(void* comm, void* stream, int64_t ticket);
int ggs_comm_size(void* comm, int32_t* nranks, int32_t* rank);
/* What RCCL itself reports for `comm` (ncclCommCount, ncclCommUserRank,
 * ncclCommCuDevice); GGS_EINVAL for a loopback communicator (no RCCL). */
int ggs_comm_info(void* comm, int32_t* nranks, int32_t* rank, int32_t* device);
/* Provenance of the runtimes in this process, as JSON into buf[cap]: the HIP
 * runtime libggs is bound to (path, version), the RCCL libggs loaded (path,
 * version; null before the first communicator) and whether both come from one
 * directory.  RCCL is always loaded from the HIP runtime's directory and a mixed
 * pair is refused (ggs_comm_* fail with GGS_ENODEV).  Returns 0, or the buffer
 * size needed (> 0) when cap is too small. */
int ggs_runtime_info(char* buf, int32_t cap);
void ggs_comm_destroy(void* comm);
/* Single-process communicators over the n listed devices (ncclCommInitAll; no id
 * exchange): comms[i] is rank i on devices[i].  The host API uses this for its
 * own multi-device fan-out (ggs_fitness with n_devices > 1). */
int ggs_comm_init_local(int32_t n, const int32_t* devices, void** comms);
/* Loopback group (test rig, no RCCL): n communicators on ONE device of this
 * process acting as ranks 0..n-1 of one job, so a one-GPU box runs the sharded
 * paths (rank != 0, uneven and empty shards, ggs_ga_set_comm's fingerprint
 * check).  Device all-gathers are matched by call order: every rank calls once
 * per gather (lockstep; a second call before all ranks called fails), the last
 * call enqueues the shard copies on every rank's stream — so d_recv on rank r's
 * stream is defined only after EVERY rank has called for that gather (work a
 * rank queues on its stream before then does not see it).  A HIP failure while
 * the last call enqueues poisons the group (every later call fails).  Host all-gathers /
 * barriers block until all n ranks (on their own host threads) arrived, at most
 * GGS_LOOPBACK_TIMEOUT_S seconds (default 60), then fail. */
int ggs_comm_init_loopback(int32_t device, int32_t n, void** comms);
/* Host-pointer all-gather (synchronous): recv[r*count + i] = rank r's send[i].
 * Staged through the communicator's own device buffer and stream; for small
 * control values (timings, session fingerprints).  count = 0: a barrier. */
int ggs_comm_allgather_host(void* comm, const float* send, float* recv, int64_t count);
/* Returns once every rank of `comm` has called it (host-side barrier). */
int ggs_comm_barrier(void* comm);

/* ---- per-kernel timing (HIP events on the launch stream) --------------------
 * When enabled, every launch of "prep", "raster" and "finalize" is bracketed
 * by hipEvents; ggs_profile_read synchronises those events and returns the
 * accumulated milliseconds and launch count for the named kernel (a finalize
 * folded into the raster counts as raster time, no finalize launch). */
int ggs_profile_enable(int32_t on);
int ggs_profile_read(const char* kernel, double* total_ms, int64_t* launches);
void ggs_profile_reset(void);

#ifdef __cplusplus
}
#endif
#endif /* GGS_H_ */
