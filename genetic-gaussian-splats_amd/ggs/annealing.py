"""Simulated annealing around the MI355X evaluator (SURVEY.md §8f next #4;
BASELINE configs[4]: run_sags.py, 2048², 4096 splats, 8 tries per iteration).

Restates annealing.py:19-190 with one change of *schedule*, not of result:
the reference evaluates its ``tries_per_iter`` neighbours one launch at a time
because each try mutates the CURRENT state, which an acceptance changes.  The
mutation draws do not depend on the state (``NumpyDraws`` draws fixed-size
arrays; the reference's torch stream is separate from the Python stream the
acceptance test uses), so here the remaining tries of an iteration are
mutated from the current state and evaluated in ONE batched libggs launch;
the acceptance test then walks them in order, and on the first acceptance the
rest of the batch is discarded and re-mutated from the new state with the
same draws.  The accepted sequence, the acceptance draws consumed, the best
individual and the curves are exactly the sequential loop's
(tests/test_sa.py replays the reference's recorded draws through both widths).

``speculate`` bounds the batch width: None adapts it to the observed
acceptance rate (wide when moves are rarely accepted — the common case at low
temperature — narrow when most are).

With the device backend and no explicit draws the loop itself runs on the GPU
(``ggs_sa_run``, ``loop="device"``, the default there): a round mutates the next
tries from the current state — across iteration boundaries, so a round can hold
more neighbours than one iteration has tries when acceptances are rare —
evaluates them in one launch, and a one-workgroup kernel walks them in order
with the same Metropolis test and installs the accepted neighbour; the host
syncs once per batch of rounds.  Its acceptance uniforms are Philox keyed by
(seed, iteration, try) (``ga_device.PhiloxAcceptDraws``), so ``loop="host"``
with the device backend replays the same trajectory on the host
(tests/test_gpu_ga.py).
"""
from __future__ import annotations

import math
import time
from typing import Callable, Optional

import numpy as np

from .ga import (NumpyDraws, mutate_batch, new_population, save_curves_csv, save_frame_png,
                 save_loss_curve_png)


def temp_schedule(kind: str, T0: float, i: int, total: int) -> float:
    """annealing.py:29-44."""
    p = i / max(1, total)
    if kind == "linear":
        return max(1e-12, T0 * (1.0 - p))
    if kind == "cosine":
        return max(1e-12, T0 * 0.5 * (1.0 + math.cos(math.pi * p)))
    if kind == "log":
        return max(1e-12, T0 / (1.0 + math.log(1.0 + 9.0 * i)))
    if kind == "cauchy":
        return max(1e-12, T0 / (1.0 + i))
    r = 0.01 ** (1.0 / max(1, total))                       # "exp" and the fallback
    return T0 * (r ** i)


def _slice(d, a: int, b: int):
    return {k: np.asarray(v)[a:b] for k, v in d.items()}


def simulated_annealing(target_img_uint8, H: int, W: int, device, n_splats: int, mutpb: float,
                        mut_sigma_max: dict, mut_sigma_min: dict, sigma_schedule: str,
                        min_scale_splats: float, max_scale_splats: float, k_sigma: float,
                        mask_strength: float, boost_only: bool, iterations: int, temp0: float,
                        temp_schedule: str, tries_per_iter: int = 1, save_video: bool = False,
                        frame_every: int = 10_000, video_dir: str = "", prefix: str = "sa",
                        loss_png_path: str = "", loss_csv_path: str = "",
                        loss_log_y: bool = False, *, seed: Optional[int] = None, draws=None,
                        evaluate: Optional[Callable[[np.ndarray], np.ndarray]] = None,
                        init_individual: Optional[np.ndarray] = None, progress: bool = True,
                        return_state: bool = False, speculate: Optional[int] = None,
                        backend: str = "auto", incremental: bool = False, loop: str = "auto",
                        chunk: int = 256):
    """annealing.py:47-190 → (best individual [N, 9] float32, best energy).

    Keyword-only hooks as ggs.ga.genetic_approx (``seed``, ``draws`` — a source
    with ``mutation(n, N, mutpb)`` and ``accept()`` —, ``evaluate``,
    ``init_individual``, ``return_state``) plus ``speculate`` (see module doc)
    and ``backend``: "host" (numpy mutation + one libggs launch per batch),
    "device" (current state resident in HBM, mutation in-kernel: Philox keyed by
    (seed, iteration, try), or the explicit ``draws``; ggs/ga_device.DeviceSA) or
    "auto" (device unless an ``evaluate`` hook is given).  ``incremental``
    (device backend): re-rasterise only the strips the changed splats touch
    (bit-identical results; off by default — the double ``wrap_angle`` of
    genetic.py:71 + utils.py:43 moves many θ by an ulp on every mutation, so
    most strips are dirty anyway and the bookkeeping costs more than it saves,
    DESIGN.md §8).  ``loop``: "device" (the whole iteration on the GPU, see the
    module doc; device backend, Philox draws), "host" (acceptance test in Python)
    or "auto" (device when possible).  ``chunk``: iterations per ``ggs_sa_run``
    call in the device loop (progress bar / interrupt granularity; video frames
    fall on chunk ends)."""
    from .mask import compute_importance_mask, prepare_target
    from .ga import resolve_seed
    seed = resolve_seed(seed)                                # run_sags.py:26-27 seeds `random`
    sched = temp_schedule
    t = prepare_target(target_img_uint8, H, W)                       # annealing.py:87
    imp_mask = compute_importance_mask(t, H, W, edge_scales=(1, 2, 4), w_edge=0.7, w_var=0.3,
                                       gamma=0.7, floor=0.15, smooth=3,
                                       strength=mask_strength)        # annealing.py:89-94
    if backend == "auto":
        backend = "device" if evaluate is None else "host"
    if evaluate is None:
        from . import api

        def evaluate(G):
            return api.fitness(G, t, H, W, k_sigma, weight_mask=imp_mask, boost_only=boost_only,
                               device=device)
    explicit = draws is not None
    if loop == "auto":
        loop = "device" if backend == "device" and not explicit else "host"
    if loop not in ("host", "device"):
        raise ValueError(f"loop must be 'auto', 'host' or 'device', got {loop!r}")
    if loop == "device" and (backend != "device" or explicit):
        raise ValueError("loop='device' needs backend='device' and the in-kernel (Philox) draws")
    if draws is None:
        if backend == "device":          # Philox mutation in-kernel; acceptance as ggs_sa_run
            from .ga_device import PhiloxAcceptDraws
            draws = PhiloxAcceptDraws(seed)
        else:
            draws = NumpyDraws(seed)
    curr = (np.array(init_individual, np.float32, copy=True) if init_individual is not None else
            new_population(1, n_splats, H, W, min_scale_splats, max_scale_splats,
                           np.random.default_rng(seed))[0])
    N = curr.shape[0]
    tries = max(0, int(tries_per_iter))
    if backend == "device":
        cap = max(1, tries)
        if loop == "device":             # a round may span iterations: size it to fill the GPU
            cap = max(1, int(speculate)) if speculate is not None else device_loop_width(H, W, tries)
        prop = _DeviceProposer(t, imp_mask, curr, cap, mutpb, mut_sigma_max,
                               mut_sigma_min, sigma_schedule, min_scale_splats, max_scale_splats,
                               k_sigma, boost_only, seed, incremental, device)
    elif backend == "host":
        prop = _HostProposer(curr, evaluate, iterations, sigma_schedule, mut_sigma_max,
                             mut_sigma_min, mutpb, H, W, min_scale_splats, max_scale_splats)
    else:
        raise ValueError(f"backend must be 'auto', 'host' or 'device', got {backend!r}")
    try:
        curr_fit = prop.init_fit                                           # annealing.py:99-101
        best_fit = curr_fit
        curves = {"best": [best_fit], "current": [curr_fit]}
        pad = len(str(iterations))
        if save_video:
            save_frame_png(0, prop.best(), pad, prefix, video_dir, H, W, k_sigma, device, save_video)

        if loop == "device":
            best_fit, curr_fit, stats = _device_loop(
                prop.sa, curves, iterations, tries, sched, temp0, 0 if speculate is None else
                max(1, int(speculate)), chunk, progress, save_video, frame_every,
                lambda i: save_frame_png(i, prop.best(), pad, prefix, video_dir, H, W, k_sigma,
                                         device, save_video))
            best, curr = prop.best(), prop.current()
            stats.update(prop.stats())
            return _finish(best, best_fit, curr, curr_fit, curves, stats, prefix, loss_png_path,
                           loss_csv_path, loss_log_y, return_state)
        acc_rate = 0.0                 # EWMA of the per-try acceptance rate
        stats = {"evaluated": 0, "tries": 0, "launches": 0, "accepted": 0}
        t_loop = time.perf_counter()
        bar = range(iterations)
        if progress:
            try:
                from tqdm.auto import tqdm
                bar = tqdm(bar, desc="SA iterations", leave=True)
            except ImportError:
                pass
        try:
            for it in bar:
                T = _T(sched, temp0, it, iterations)
                accepted_any = False
                e_curr = float(curr_fit)
                d = draws.mutation(tries, N, mutpb) if tries and (explicit or backend == "host") \
                    else None
                k = 0
                while k < tries:
                    if speculate is not None:
                        w = max(1, int(speculate))
                    else:
                        w = tries if acc_rate < 1.0 / tries else max(1, int(round(1.0 / acc_rate)))
                    w = min(w, tries - k)
                    e = prop.propose(it, iterations, k, w, None if d is None else _slice(d, k, k + w))
                    stats["evaluated"] += w
                    stats["launches"] += 1
                    for j in range(w):
                        e_new = float(e[j])
                        dE = e_new - e_curr                                # annealing.py:133
                        acc = dE <= 0.0
                        if not acc and T > 0.0:
                            u = draws.accept_at(it, k) if hasattr(draws, "accept_at") else \
                                draws.accept()
                            acc = u < math.exp(-dE / T)                    # annealing.py:140-142
                        k += 1
                        acc_rate = 0.9 * acc_rate + 0.1 * float(acc)
                        if acc:
                            curr_fit = e_new
                            e_curr = curr_fit
                            accepted_any = True
                            stats["accepted"] += 1
                        new_best = e_curr + 1e-12 < best_fit               # annealing.py:148-150
                        if new_best:
                            best_fit = e_curr
                        if acc or new_best:
                            prop.commit(j if acc else -1, new_best)
                        if acc:
                            break              # the rest of the batch came from the old state
                stats["tries"] += tries
                curves["best"].append(best_fit)
                curves["current"].append(float(curr_fit))
                if save_video and (it + 1) % max(1, frame_every) == 0:
                    save_frame_png(it + 1, prop.best(), pad, prefix, video_dir, H, W, k_sigma,
                                   device, save_video)
                if hasattr(bar, "set_postfix"):
                    bar.set_postfix(best_mse=f"{best_fit:.6f}", curr_mse=f"{float(curr_fit):.6f}",
                                    T=f"{T:.4g}", accepted="Y" if accepted_any else "N")
        except KeyboardInterrupt:
            print("\n[Interrupted] Returning current best…", flush=True)
        finally:
            if hasattr(bar, "close"):
                bar.close()
        stats["loop_s"] = time.perf_counter() - t_loop
        best, curr = prop.best(), prop.current()
        stats.update(prop.stats())
    finally:
        prop.close()
    return _finish(best, best_fit, curr, curr_fit, curves, stats, prefix, loss_png_path,
                   loss_csv_path, loss_log_y, return_state)


def device_loop_width(H: int, W: int, tries: int) -> int:
    """Neighbour capacity of a device-loop round: enough 16x128 strips to fill the
    GPU's 3,072 raster wave slots several times over (2048^2: 16 neighbours of
    2,048 strips; 512^2: 64 of 256), never below one iteration's tries."""
    strips = 4 * (-(-W // 64)) * (-(-H // 128))
    return max(1, tries, min(64, -(-32768 // strips)))


def _device_loop(sa, curves, iterations, tries, sched, temp0, width, chunk, progress, save_video,
                 frame_every, save_frame):
    """annealing.py:117-172 on the GPU (ggs_sa_run), ``chunk`` iterations per call."""
    bar = None
    if progress:
        try:
            from tqdm.auto import tqdm
            bar = tqdm(total=iterations, desc="SA iterations", leave=True)
        except ImportError:
            pass
    st = sa.loop_state()
    it = 0
    t0 = time.perf_counter()
    try:
        while it < iterations:
            n = min(max(1, int(chunk)), iterations - it)
            if save_video:               # frames fall on chunk ends
                fe = max(1, frame_every)
                n = min(n, fe - it % fe)
            if tries:
                temps = [_T(sched, temp0, i, iterations) for i in range(it, it + n)]
                cv = sa.run(it, temps, iterations, tries, width)
                curves["best"].extend(cv[:, 0].tolist())
                curves["current"].extend(cv[:, 1].tolist())
                st = sa.loop_state()
            else:                        # no tries: the state never moves
                curves["best"].extend([st["best_fit"]] * n)
                curves["current"].extend([st["current_fit"]] * n)
            it += n
            if save_video and it % max(1, frame_every) == 0:
                save_frame(it)
            if bar is not None:
                bar.update(n)
                bar.set_postfix(best_mse=f"{st['best_fit']:.6f}", curr_mse=f"{st['current_fit']:.6f}",
                                T=f"{_T(sched, temp0, it - 1, iterations):.4g}")
    except KeyboardInterrupt:
        print("\n[Interrupted] Returning current best…", flush=True)
    finally:
        if bar is not None:
            bar.close()
    stats = {"evaluated": st["evaluated"], "tries": it * tries, "launches": st["rounds"],
             "accepted": st["accepted"], "loop_s": time.perf_counter() - t0}
    return st["best_fit"], st["current_fit"], stats


def _finish(best, best_fit, curr, curr_fit, curves, stats, prefix, loss_png_path, loss_csv_path,
            loss_log_y, return_state):
    try:                                                                   # annealing.py:174-188
        save_loss_curve_png(curves, loss_png_path, title=f"{prefix} energy (MSE)",
                            xlabel="Iteration", ylabel="MSE", log_y=loss_log_y, dpi=144)
        save_curves_csv(curves, loss_csv_path)
        if loss_png_path:
            print(f"Saved loss plot to {loss_png_path}")
        if loss_csv_path:
            print(f"Saved loss CSV to {loss_csv_path}")
    except Exception as e:  # noqa: BLE001 — as the reference
        print(f"[warn] Could not save SA curves: {e}")
    if return_state:
        return best, float(best_fit), {"current": curr, "current_fit": curr_fit,
                                       "curves": curves, "stats": stats}
    return best, float(best_fit)


_T = temp_schedule


class _HostProposer:
    """Neighbours mutated by ggs.ga.mutate_batch, evaluated by ``evaluate``."""

    def __init__(self, curr, evaluate, iterations, schedule, sig_max, sig_min, mutpb, H, W,
                 min_s, max_s):
        self.curr, self.evaluate = curr, evaluate
        self.args = (iterations, schedule, sig_max, sig_min, mutpb, H, W, min_s, max_s)
        self.init_fit = float(np.asarray(evaluate(curr[None]), np.float32)[0])
        self._best = curr.copy()
        self.nb = None

    def propose(self, it, total, first_try, w, d):
        total_, sched, smax, smin, mutpb, H, W, lo, hi = self.args
        self.nb = mutate_batch(np.repeat(self.curr[None], w, axis=0), d, it, total_, sched, smax,
                               smin, mutpb, H, W, lo, hi)
        return np.asarray(self.evaluate(self.nb), np.float32)

    def commit(self, j, update_best):
        if j >= 0:
            self.curr = self.nb[j].copy()
        if update_best:
            self._best = self.curr.copy()

    def best(self):
        return self._best.copy()

    def current(self):
        return self.curr.copy()

    def stats(self):
        return {}

    def close(self):
        pass


class _DeviceProposer:
    """Neighbours mutated and evaluated on the GPU (ggs_sa_*)."""

    def __init__(self, t, mask, curr, max_tries, mutpb, sig_max, sig_min, schedule, min_s, max_s,
                 k_sigma, boost_only, seed, incremental=False, device=None):
        from . import api
        from .ga_device import DeviceSA
        self.sa = DeviceSA(t, mask, curr, max_tries=max_tries, mutpb=mutpb, mut_sigma_max=sig_max,
                           mut_sigma_min=sig_min, schedule=schedule, min_scale_splats=min_s,
                           max_scale_splats=max_s, k_sigma=k_sigma, boost_only=boost_only,
                           seed=int(seed) & (2**64 - 1), incremental=incremental,
                           device=api.device_index(device))
        self.init_fit = float(self.sa.init_fit)

    def stats(self):
        return self.sa.stats()

    def propose(self, it, total, first_try, w, d):
        return self.sa.propose(it, total, first_try, w, d)

    def commit(self, j, update_best):
        self.sa.commit(j, update_best)

    def best(self):
        return self.sa.read()[1]

    def current(self):
        return self.sa.read()[0]

    def close(self):
        self.sa.close()
