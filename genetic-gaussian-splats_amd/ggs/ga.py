"""Batched genetic algorithm around the MI355X evaluator.

Restates the reference's GA layer over whole populations instead of one
individual at a time:

* ``new_population``          population.py:20-46   (numpy RNG)
* ``tournament`` / ``crossover`` / ``mutate_batch``
                              genetic.py:8-21, 32-91 (every candidate of a
                              generation in one set of numpy array ops)
* ``build_mut_sigma`` / ``wrap_angle`` / ``clamp_genome``   utils.py:10-45
* ``genetic_approx``          algorithm.py:17-195    (same signature; one
                              libggs fitness launch per generation)

Randomness comes from a *draw source*.  ``NumpyDraws`` (default) samples the
same distributions as the reference's torch / Python RNG calls, in batches.
The operators consume the draws with exactly the reference's arithmetic
(float32, same operation order), so given the reference's own draws they
reproduce its results bit for bit — tests/test_ga.py replays draws recorded
from the reference (tests/golden/make_golden_ga.py) to prove it.

Two deliberate differences, both in what is evaluated, not in any result: the
reference re-evaluates the elites every generation (algorithm.py:134-137); the
evaluator is deterministic (same genome → same bits, tests/test_gpu_parity.py),
so their fitness is carried over instead of recomputed.  And it evaluates all
P offspring (algorithm.py:123-126) although only offspring[:P - elite_k] survive
(:140-141) and nothing reads the others' fitness; they are bred (their draws keep
the trajectory) but not evaluated, so an ``evaluate`` hook sees P - elite_k rows
per generation.  The returned values are identical.
"""
from __future__ import annotations

import csv
import math
import os
import random
import statistics
from typing import Callable, Dict, Optional, Sequence, Tuple

import numpy as np

_f32 = np.float32
PI32 = _f32(np.pi)
TWO_PI32 = _f32(2 * np.pi)


# ---------------------------------------------------------------------------
# utils.py:10-45
# ---------------------------------------------------------------------------
def wrap_angle(theta: np.ndarray) -> np.ndarray:
    """utils.py:10-11: (θ + π) mod 2π − π in float32 (Python-style modulo)."""
    return np.remainder(theta + PI32, TWO_PI32) - PI32


def anneal_factor(gen: int, total: int, kind: str) -> float:
    """utils.py:14-27."""
    g = max(0, min(gen, total))
    p = g / max(1, total)
    if kind == "cosine":
        raw = 0.5 * (1.0 + math.cos(math.pi * p))
    elif kind == "linear":
        raw = 1.0 - p
    elif kind == "exp":
        decay = 0.2 ** (1.0 / max(1, total))
        raw = decay ** g
    else:
        raw = 1.0 - p
    return max(0.0, raw)


def build_mut_sigma(gen: int, total_gens: int, kind: str, mut_sigma_max: Dict[str, float],
                    mut_sigma_min: Dict[str, float]) -> Dict[str, float]:
    """utils.py:30-32."""
    f = anneal_factor(gen, total_gens, kind)
    return {k: mut_sigma_min[k] + f * (mut_sigma_max[k] - mut_sigma_min[k]) for k in mut_sigma_max}


def scale_log_bounds(H: int, W: int, min_scale_splats: float,
                     max_scale_splats: float) -> Tuple[np.float32, np.float32]:
    """utils.py:38-39: log of the float32 scale bounds."""
    max_side = float(max(H, W))
    return (np.log(_f32(min_scale_splats)).astype(np.float32),
            np.log(_f32(max_scale_splats * max_side)).astype(np.float32))


def clamp_genome(G: np.ndarray, H: int, W: int, min_scale_splats: float,
                 max_scale_splats: float) -> np.ndarray:
    """utils.py:35-45 on [..., N, 9] in place."""
    lo, hi = scale_log_bounds(H, W, min_scale_splats, max_scale_splats)
    G[..., 0:2] = np.clip(G[..., 0:2], _f32(0.0), _f32(1.0))
    G[..., 2] = np.clip(G[..., 2], lo, hi)
    G[..., 3] = np.clip(G[..., 3], lo, hi)
    G[..., 4] = wrap_angle(G[..., 4])
    G[..., 5:9] = np.clip(G[..., 5:9], _f32(0.0), _f32(255.0))
    return G


# ---------------------------------------------------------------------------
# draw sources
# ---------------------------------------------------------------------------
def resolve_seed(seed: Optional[int] = None) -> int:
    """An explicit seed, or — when None — one drawn from Python's global ``random``
    state, so that ``random.seed(SEED)`` in the reference's entry scripts
    (run_ggs.py:25-28, run_sags.py:26-27) makes a run repeatable here too."""
    return int(seed) if seed is not None else random.getrandbits(63)


class NumpyDraws:
    """Batched draws with the distributions of the reference's RNG calls.  With
    ``seed=None`` the generator is seeded from Python's ``random`` at first use
    (``resolve_seed``), not at construction: module-level sources made at import
    time still follow a later ``random.seed``."""

    def __init__(self, seed: Optional[int] = None):
        self._seed = seed
        self._rng = None

    @property
    def rng(self) -> np.random.Generator:
        if self._rng is None:
            self._rng = np.random.default_rng(resolve_seed(self._seed))
        return self._rng

    def tournament(self, P: int, k: int) -> np.ndarray:           # random.randrange (genetic.py:11)
        return self.rng.integers(0, P, (P, k))

    def shuffle(self, P: int) -> np.ndarray:                       # random.shuffle (algorithm.py:90)
        return self.rng.permutation(P)

    def uniform(self, n: int) -> np.ndarray:                       # random.random (algorithm.py:97)
        return self.rng.random(n)

    def crossover_masks(self, n: int, N: int) -> np.ndarray:       # torch.rand((N,1)) (genetic.py:18)
        return self.rng.random((n, N, 1), dtype=np.float32)

    def mutation(self, P: int, N: int, mutpb: float) -> Dict[str, np.ndarray]:
        """genetic.py:37-91: mask uniforms, one-true fallbacks, normals, swap."""
        r = self.rng
        u = lambda *s: r.random((P,) + s, dtype=np.float32)      # noqa: E731
        n = lambda *s: r.standard_normal((P,) + s, dtype=np.float32)  # noqa: E731
        return {
            "u_xy": u(N, 2), "u_ab": u(N, 2), "u_t": u(N, 1), "u_rgb": u(N, 1), "u_a": u(N, 1),
            "k_color": r.integers(0, 2 * N, P), "k_xy": r.integers(0, 2 * N, P),
            "k_ab": r.integers(0, 2 * N, P), "k_t": r.integers(0, N, P),
            "n_xy": n(N, 2), "n_ab": n(N, 2), "n_t": n(N, 1), "n_rgba": n(N, 4),
            "swap_i": r.integers(0, max(N - 1, 1), P), "swap_pick": np.full(P, -1),
            "swap_u": r.random(P),
        }

    def accept(self) -> float:                                     # random.random (annealing.py:142)
        return float(self.rng.random())

    def generation(self, cx: np.ndarray, n_off: int, N: int, mutpb: float):
        """Crossover masks for the crossing pairs + mutation draws for the offspring."""
        return self.crossover_masks(int(cx.sum()), N), self.mutation(n_off, N, mutpb)


# ---------------------------------------------------------------------------
# population.py:20-46
# ---------------------------------------------------------------------------
def new_population(batch_size: int, n_splats: int, H: int, W: int, min_scale_splats: float,
                   max_scale_splats: float, rng: Optional[np.random.Generator] = None) -> np.ndarray:
    """[B, N, 9] axes-angle genomes with population.py's distributions."""
    rng = rng if rng is not None else np.random.default_rng(resolve_seed())
    B, N = batch_size, n_splats
    s_lo, s_hi = float(min_scale_splats), float(max_scale_splats * float(max(H, W)))

    def log_scales(m, conc=8.0, eps=1e-6):                     # population.py:6-15
        u = rng.beta(m * max(conc, eps) + eps, (1 - m) * max(conc, eps) + eps, (B, N, 1))
        return np.log((s_lo + u.astype(np.float32) * _f32(s_hi - s_lo)).astype(np.float32))

    G = np.concatenate([
        rng.random((B, N, 2), dtype=np.float32),
        log_scales(0.4), log_scales(0.6),
        rng.uniform(-np.pi, np.pi, (B, N, 1)).astype(np.float32),
        rng.uniform(0.0, 256.0, (B, N, 3)).astype(np.float32),
        rng.uniform(180.0, 256.0, (B, N, 1)).astype(np.float32),
    ], axis=-1).astype(np.float32)
    G[..., 0:2] = np.clip(G[..., 0:2], 0.0, 1.0)
    G[..., 5:9] = np.clip(G[..., 5:9], 0.0, 255.0)
    return G


# ---------------------------------------------------------------------------
# genetic.py operators, batched
# ---------------------------------------------------------------------------
def tournament(fits: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """genetic.py:8-14 for every selection at once: idx [P, k] drawn indices;
    the winner is the first drawn index with the smallest fitness."""
    return idx[np.arange(len(idx)), np.argmin(np.asarray(fits)[idx], axis=1)]


def crossover(a: np.ndarray, b: np.ndarray, u: np.ndarray, p: float = 0.5):
    """genetic.py:17-21 batched: a, b [n, N, C], u [n, N, 1] uniforms."""
    m = u < _f32(p)
    return np.where(m, a, b), np.where(m, b, a)


def _ensure_one_true(m: np.ndarray, k: np.ndarray) -> np.ndarray:
    """genetic.py:24-29 per individual: if no flag is set, set flat index k."""
    flat = m.reshape(len(m), -1)
    none = ~flat.any(axis=1)
    rows = np.nonzero(none)[0]
    flat[rows, k[rows]] = True
    return flat.reshape(m.shape)


def mutate_batch(G: np.ndarray, d: Dict[str, np.ndarray], gen: int, total_gens: int,
                 schedule: str, mut_sigma_max: Dict[str, float], mut_sigma_min: Dict[str, float],
                 mutpb: float, H: int, W: int, min_scale_splats: float,
                 max_scale_splats: float) -> np.ndarray:
    """genetic.py:32-91 for a batch [P, N, 9] (in place; returns G)."""
    SIG = build_mut_sigma(gen, total_gens, schedule, mut_sigma_max, mut_sigma_min)
    P, N = G.shape[:2]
    p = _f32(mutpb)
    m_xy = d["u_xy"] < p
    m_ab = d["u_ab"] < p
    m_t = d["u_t"] < p
    pair = _ensure_one_true(np.concatenate([d["u_rgb"] < p, d["u_a"] < p], axis=2), d["k_color"])
    m_rgba = np.concatenate([np.repeat(pair[..., 0:1], 3, axis=2), pair[..., 1:2]], axis=2)
    m_xy = _ensure_one_true(m_xy, d["k_xy"])
    m_ab = _ensure_one_true(m_ab, d["k_ab"])
    m_t = _ensure_one_true(m_t, d["k_t"])

    G[..., 0:2] += (d["n_xy"] * _f32(SIG["xy"])) * m_xy.astype(np.float32)
    sig_ab = np.array([SIG["alog"], SIG["blog"]], np.float32)
    G[..., 2:4] += (d["n_ab"] * sig_ab) * m_ab.astype(np.float32)
    G[..., 4:5] += (d["n_t"] * _f32(SIG["theta"])) * m_t.astype(np.float32)
    G[..., 4] = wrap_angle(G[..., 4])
    sig_rgba = np.array([SIG["rgb"], SIG["rgb"], SIG["rgb"], SIG["alpha"]], np.float32)
    G[..., 5:9] += (d["n_rgba"] * sig_rgba) * m_rgba.astype(np.float32)
    clamp_genome(G, H, W, min_scale_splats, max_scale_splats)

    if N >= 2:                                                    # genetic.py:79-91
        i = np.asarray(d["swap_i"], np.int64)
        rows = np.arange(P)
        size = np.exp(G[..., 2]) * np.exp(G[..., 3])
        cand = (np.arange(N)[None, :] > i[:, None]) & (size > size[rows, i][:, None])
        count = cand.sum(axis=1)
        pick = np.asarray(d["swap_pick"], np.int64).copy()
        fresh = pick < 0
        pick[fresh] = np.minimum((np.asarray(d["swap_u"])[fresh] * count[fresh]).astype(np.int64),
                                 np.maximum(count[fresh] - 1, 0))
        has = count > 0
        csum = np.cumsum(cand, axis=1)
        j = np.argmax(cand & (csum == (pick + 1)[:, None]), axis=1)   # (pick+1)-th candidate
        r = rows[has]
        gi, gj = G[r, i[has]].copy(), G[r, j[has]].copy()
        G[r, i[has]] = gj
        G[r, j[has]] = gi
    return G


# ---------------------------------------------------------------------------
# algorithm.py:17-195
# ---------------------------------------------------------------------------
def next_generation(pop: np.ndarray, fits: np.ndarray, draws, gen: int, generations: int,
                    tour_k: int, cxpb: float, mutpb: float, mut_sigma_max, mut_sigma_min,
                    schedule: str, H: int, W: int, min_scale_splats: float,
                    max_scale_splats: float) -> np.ndarray:
    """algorithm.py:86-120: selection, crossover and mutation → offspring [P, N, C]."""
    P = len(pop)
    parents = tournament(fits, draws.tournament(P, tour_k))
    parents = parents[draws.shuffle(P)]
    npairs = (P + 1) // 2
    a_idx = parents[0::2][:npairs]
    b_idx = parents[(np.arange(npairs) * 2 + 1) % P]
    cx = draws.uniform(npairs) < cxpb
    cxu, mut = draws.generation(cx, P, pop.shape[1], mutpb)
    c1 = pop[a_idx].copy()
    c2 = pop[b_idx].copy()
    if cx.any():
        c1[cx], c2[cx] = crossover(pop[a_idx[cx]], pop[b_idx[cx]], cxu)
    off = np.empty((2 * npairs,) + pop.shape[1:], pop.dtype)
    off[0::2], off[1::2] = c1, c2
    off = np.ascontiguousarray(off[:P])
    return mutate_batch(off, mut, gen, generations, schedule, mut_sigma_max, mut_sigma_min,
                        mutpb, H, W, min_scale_splats, max_scale_splats)


def _render_best_u8(best: np.ndarray, H: int, W: int, k_sigma: float, device=None) -> np.ndarray:
    """utils.py:48-58: render one axes-angle genome to uint8 [H, W, 3]."""
    from . import api
    img = api.render(api.encode(best[None]), H, W, k_sigma=k_sigma, device=device)[0]
    return (np.clip(img, 0, 1) * 255.0).astype(np.uint8)


def save_frame_png(gen: int, ind, pad: int, prefix: str, video_dir: str, H: int, W: int,
                   k_sigma: float, device=None, save_video: bool = True) -> None:
    """utils.py:61-69."""
    if not save_video:
        return
    from PIL import Image
    fname = f"{prefix}_{gen:0{pad}d}.png"
    Image.fromarray(_render_best_u8(np.asarray(ind, np.float32), H, W, k_sigma, device)).save(
        os.path.join(video_dir, fname))


def save_curves_csv(curves: Dict[str, Sequence[float]], out_csv_path: str) -> None:
    """utils.py:133-151: gen,<key1>,<key2>,..."""
    if not out_csv_path:
        return
    d = os.path.dirname(out_csv_path)
    if d:
        os.makedirs(d, exist_ok=True)
    keys = list(curves.keys())
    lens = [len(v) for v in curves.values() if len(v) > 0]
    if not lens:
        print("[warn] No values to save to CSV")
        return
    with open(out_csv_path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["gen"] + keys)
        for i in range(lens[0]):
            w.writerow([i] + [curves[k][i] if i < len(curves[k]) else "" for k in keys])


def save_loss_curve_png(curves, out_path: str, title: str = "GA fitness over generations",
                        xlabel: str = "Generation", ylabel: str = "MSE", log_y: bool = False,
                        dpi: int = 144) -> None:
    """utils.py:85-130: one line per named curve against its index, written as a
    PNG.  Same contract as the reference: nothing when out_path is empty; a
    warning and no file without matplotlib or without any values; ValueError when
    the non-empty curves differ in length."""
    if not out_path:
        return
    try:
        import matplotlib
        matplotlib.use("Agg")
        from matplotlib.figure import Figure
    except Exception as e:  # noqa: BLE001 — the reference degrades to a warning too
        print(f"[warn] matplotlib not available, cannot save plot: {e}")
        return
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    series = {k: list(v) for k, v in curves.items() if len(v)}
    if not series:
        print("[warn] No values to plot")
        return
    lengths = {k: len(v) for k, v in series.items()}
    n = next(iter(lengths.values()))
    bad = [k for k, m in lengths.items() if m != n]
    if bad:
        raise ValueError(f"Curve '{bad[0]}' length {lengths[bad[0]]} does not match others {n}")
    fig = Figure()
    ax = fig.add_subplot()
    x = np.arange(n)
    for name, ys in series.items():
        ax.plot(x, ys, label=name)
    ax.set(title=title, xlabel=xlabel, ylabel=ylabel)
    if log_y:
        ax.set_yscale("log")
    ax.grid(True, which="both", alpha=0.3)
    ax.legend()
    fig.tight_layout()
    fig.savefig(out_path, dpi=dpi)


def genetic_approx(target_img_uint8, H: int, W: int, device, pop_size: int, n_splats: int,
                   generations: int, tour_k: int, elite_k: int, cxpb: float, mutpb: float,
                   mut_sigma_max: dict, mut_sigma_min: dict, schedule: str,
                   min_scale_splats: float, max_scale_splats: float, k_sigma: float,
                   mask_strength: float, boost_only: bool, save_video: bool = False,
                   frame_every: int = 5000, video_dir: str = "", prefix: str = "ga",
                   loss_png_path: str = "", loss_csv_path: str = "", loss_log_y: bool = False,
                   *, seed: Optional[int] = None, draws=None,
                   evaluate: Optional[Callable[[np.ndarray], np.ndarray]] = None,
                   init_population: Optional[np.ndarray] = None, progress: bool = True,
                   return_state: bool = False, backend: str = "auto", chunk: int = 50):
    """algorithm.py:17-195 → (best individual [N, 9] float32, best fitness).

    Extra keyword-only hooks: ``seed`` / ``draws`` (draw source), ``evaluate``
    (population [M,N,9] → fitness [M]: the initial population, then the P -
    elite_k surviving offspring of each generation; default: one libggs launch
    with the importance mask), ``init_population``, ``return_state`` (also return the
    final population, fitnesses and curves), ``backend``: "host" (numpy
    operators, one libggs fitness launch per generation), "device" (the whole
    generation on the GPU, ggs/ga_device.py; Philox draws keyed by ``seed``, or
    the draws a ``ga_device.RecordingDraws`` holds; ``chunk`` generations per
    host call) or "auto" (device unless an ``evaluate`` or ``draws`` hook is
    given)."""
    from .mask import compute_importance_mask, prepare_target

    seed = resolve_seed(seed)                                          # run_ggs.py:25-28 seeds `random`
    t = prepare_target(target_img_uint8, H, W)                         # algorithm.py:33-39
    imp_mask = compute_importance_mask(t, H, W, edge_scales=(1, 2, 4), w_edge=0.7, w_var=0.3,
                                       gamma=0.7, floor=0.15, smooth=3,
                                       strength=mask_strength)          # algorithm.py:42-49
    if evaluate is None:
        from . import api

        def evaluate(G):
            return api.fitness(G, t, H, W, k_sigma, weight_mask=imp_mask, boost_only=boost_only,
                               device=device)
    pop = (np.array(init_population, np.float32, copy=True) if init_population is not None else
           new_population(pop_size, n_splats, H, W, min_scale_splats, max_scale_splats,
                          np.random.default_rng(seed)))
    if backend == "auto":
        backend = "device" if evaluate is None and draws is None else "host"
    if backend == "device":
        return _genetic_approx_device(t, imp_mask, pop, H, W, generations, tour_k, elite_k, cxpb,
                                      mutpb, mut_sigma_max, mut_sigma_min, schedule,
                                      min_scale_splats, max_scale_splats, k_sigma, boost_only,
                                      save_video, frame_every, video_dir, prefix, loss_png_path,
                                      loss_csv_path, loss_log_y, seed, draws, progress,
                                      return_state, chunk, device)
    if backend != "host":
        raise ValueError(f"backend must be 'host' or 'device', got {backend!r}")
    draws = draws if draws is not None else NumpyDraws(seed)
    fits = np.asarray(evaluate(pop), np.float32)

    best_idx = int(np.argmin(fits))
    best_ind = pop[best_idx].copy()
    best_fit = float(fits[best_idx])
    no_improve = 0
    fl = fits.tolist()
    curves = {"best": [best_fit], "mean": [float(sum(fl) / len(fl))], "median": [float(statistics.median(fl))]}
    pad = len(str(generations))
    if save_video:
        save_frame_png(0, best_ind, pad, prefix, video_dir, H, W, k_sigma, device, save_video)

    elite_k_actual = max(1, elite_k)
    bar = range(1, generations + 1)
    if progress:
        try:
            from tqdm.auto import tqdm
            bar = tqdm(bar, desc="GA generations", leave=True)
        except ImportError:
            pass
    try:
        for gen in bar:
            off = next_generation(pop, fits, draws, gen, generations, tour_k, cxpb, mutpb,
                                  mut_sigma_max, mut_sigma_min, schedule, H, W,
                                  min_scale_splats, max_scale_splats)
            # algorithm.py:123-126 evaluates all offspring, but only off[:keep] survive
            # (:140-141) and nothing reads the rest's fitness: evaluate the survivors
            keep = pop_size - elite_k_actual
            off_fits = (np.asarray(evaluate(off[:keep]), np.float32) if keep > 0
                        else np.zeros(0, np.float32))
            elite_idx = np.argsort(fits, kind="stable")[:elite_k_actual]     # algorithm.py:129-131
            pop = np.concatenate([pop[elite_idx], off[:keep]], axis=0)
            fits = np.concatenate([fits[elite_idx], off_fits[:keep]], axis=0)  # elites: carried over
            g = int(np.argmin(fits))
            if float(fits[g]) + 1e-10 < best_fit:                            # algorithm.py:144-150
                best_fit = float(fits[g])
                best_ind = pop[g].copy()
                no_improve = 0
            else:
                no_improve += 1
            fl = fits.tolist()
            curves["best"].append(float(best_fit))
            curves["mean"].append(float(sum(fl) / len(fl)))
            curves["median"].append(float(statistics.median(fl)))
            if save_video and gen % max(1, frame_every) == 0:
                save_frame_png(gen, best_ind, pad, prefix, video_dir, H, W, k_sigma, device, save_video)
            if hasattr(bar, "set_postfix"):
                bar.set_postfix(best_mse=f"{best_fit:.6f}", stale=no_improve,
                                sigma_fac=f"{anneal_factor(gen, generations, schedule):.3f}")
    except KeyboardInterrupt:
        print("\n[Interrupted] Returning current best individual…", flush=True)
    finally:
        if hasattr(bar, "close"):
            bar.close()

    save_loss_curve_png(curves, loss_png_path, title=f"{prefix} fitness", xlabel="Generation",
                        ylabel="MSE", log_y=loss_log_y, dpi=144)
    save_curves_csv(curves, loss_csv_path)
    if return_state:
        return best_ind, best_fit, {"population": pop, "fitness": fits, "curves": curves}
    return best_ind, best_fit


def _genetic_approx_device(t, imp_mask, pop, H, W, generations, tour_k, elite_k, cxpb, mutpb,
                           mut_sigma_max, mut_sigma_min, schedule, min_scale_splats,
                           max_scale_splats, k_sigma, boost_only, save_video, frame_every,
                           video_dir, prefix, loss_png_path, loss_csv_path, loss_log_y, seed,
                           draws, progress, return_state, chunk, device=None):
    """genetic_approx with backend="device" (ggs/ga_device.py) on the GPU
    ``device`` names (api.device_index)."""
    from . import api
    from .ga_device import run_device_ga
    pad = len(str(generations))
    every = max(1, frame_every)
    step = max(1, chunk)
    if save_video:
        step = math.gcd(step, every)                  # land on every frame generation
    bar = None
    if progress:
        try:
            from tqdm.auto import tqdm
            bar = tqdm(total=generations, desc="GA generations (device)", leave=True)
        except ImportError:
            pass
    state = {"gen": 0}

    def on_chunk(gen, ga):
        if bar is not None:
            bar.update(gen - state["gen"])
        state["gen"] = gen
        if save_video and gen % every == 0:
            st = ga.read()
            save_frame_png(gen, st["best"], pad, prefix, video_dir, H, W, k_sigma, device, save_video)
        if bar is not None:
            bar.set_postfix(sigma_fac=f"{anneal_factor(gen, generations, schedule):.3f}")

    if save_video:
        f0 = api.fitness(pop, t, H, W, k_sigma, weight_mask=imp_mask, boost_only=boost_only,
                         device=device)
        save_frame_png(0, pop[int(np.argmin(f0))], pad, prefix, video_dir, H, W, k_sigma, device,
                       save_video)
    replay = getattr(draws, "generations", None) if draws is not None else None
    try:
        st = run_device_ga(t, imp_mask, pop, generations, tour_k=tour_k, elite_k=elite_k,
                           cxpb=cxpb, mutpb=mutpb, mut_sigma_max=mut_sigma_max,
                           mut_sigma_min=mut_sigma_min, schedule=schedule,
                           min_scale_splats=min_scale_splats, max_scale_splats=max_scale_splats,
                           k_sigma=k_sigma, boost_only=boost_only,
                           seed=resolve_seed(seed) & (2**64 - 1), chunk=step, on_chunk=on_chunk,
                           draws=replay, device=api.device_index(device))
    finally:
        if bar is not None:
            bar.close()
    curves = st["curves"]
    save_loss_curve_png(curves, loss_png_path, title=f"{prefix} fitness", xlabel="Generation",
                        ylabel="MSE", log_y=loss_log_y, dpi=144)
    save_curves_csv(curves, loss_csv_path)
    best_ind, best_fit = st["best"], st["best_fit"]
    if return_state:
        return best_ind, best_fit, {"population": st["population"], "fitness": st["fitness"],
                                    "curves": curves}
    return best_ind, best_fit
