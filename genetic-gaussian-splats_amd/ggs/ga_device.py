"""Device-resident GA loop (ggs_ga_* in include/ggs.h, kernels in csrc/ggs_ga.hip).

The whole generation of algorithm.py:85-155 — selection, crossover, mutation,
fitness, elites, best individual, curves — runs on one GPU with no host round
trip; the host only enqueues.  ``DeviceGA.step(draws=...)`` accepts explicit
draws in ggs/ga.py's layout (tests/test_gpu_parity.py feeds it the same draws as
the host path and requires identical populations); ``DeviceGA.run`` uses the
in-kernel Philox stream.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import numpy as np

from . import _lib
from ._lib import GaConfig, GaDraws, check, lib

_f32p = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)
_f64p = C.POINTER(C.c_double)
SIG_KEYS = ("xy", "alog", "blog", "theta", "rgb", "alpha")
SCHEDULES = {"linear": 0, "cosine": 1, "exp": 2}


def _arr(x, dt):
    return np.ascontiguousarray(x, dtype=dt)


def _config(P, N, H, W, tour_k, elite_k, cxpb, mutpb, k_sigma, min_scale_splats,
            max_scale_splats, mask, boost_only, boost_beta, schedule, mut_sigma_max,
            mut_sigma_min, seed) -> GaConfig:
    from .ga import scale_log_bounds
    lo, hi = scale_log_bounds(H, W, min_scale_splats, max_scale_splats)
    mode = (_lib.GGS_FIT_NONE if mask is None else
            _lib.GGS_FIT_BOOST if boost_only else _lib.GGS_FIT_WEIGHTED)
    return GaConfig(P, N, H, W, tour_k, elite_k, cxpb, mutpb, k_sigma, min_scale_splats,
                    max_scale_splats, float(lo), float(hi), mode, boost_beta,
                    SCHEDULES.get(schedule, 0),
                    (C.c_double * 6)(*[mut_sigma_max[k] for k in SIG_KEYS]),
                    (C.c_double * 6)(*[mut_sigma_min[k] for k in SIG_KEYS]), seed & (2**64 - 1))


def _draws_struct(draws, keep, fields=None) -> GaDraws:
    d = GaDraws()
    for name, typ in GaDraws._fields_:
        if fields is not None and name not in fields:
            continue
        dt = np.float64 if name == "swap_u" else (np.int32 if typ is _i32p else np.float32)
        a = keep[name] = _arr(draws[name], dt)
        setattr(d, name, a.ctypes.data_as(typ))
    return d


class PhiloxAcceptDraws:
    """The device SA loop's acceptance uniforms (ggs_sa_accept_uniform: Philox keyed
    by (seed, iteration, try)) for the host loop, so a host-driven run with the
    device proposer follows the device loop's trajectory exactly."""

    def __init__(self, seed: int):
        self.seed = int(seed) & (2**64 - 1)

    def accept_at(self, it: int, k: int) -> float:
        u = C.c_double()
        check(lib.ggs_sa_accept_uniform(self.seed, int(it), int(k), C.byref(u)),
              "ggs_sa_accept_uniform")
        return u.value


MUTATION_KEYS = ("u_xy", "u_ab", "u_t", "u_rgb", "u_a", "k_color", "k_xy", "k_ab", "k_t", "n_xy",
                 "n_ab", "n_t", "n_rgba", "swap_i", "swap_pick", "swap_u")


class DeviceSA:
    """Device-resident SA state (ggs_sa_* in include/ggs.h): the current and best
    individuals live in HBM; ``propose`` returns the energies of a batch of tries."""

    def __init__(self, target, mask, init_ind, *, max_tries: int, mutpb: float,
                 mut_sigma_max: Dict[str, float], mut_sigma_min: Dict[str, float],
                 schedule: str, min_scale_splats: float, max_scale_splats: float,
                 k_sigma: float = 3.0, boost_only: bool = False, boost_beta: float = 1.0,
                 seed: int = 0, device: int = 0, incremental: bool = False):
        ind = _arr(init_ind, np.float32)
        if ind.ndim != 2 or ind.shape[1] != 9:
            raise _lib.GGSInputError("the device SA keeps an [N, 9] genome")
        self.target = _arr(target, np.float32)
        H, W = self.target.shape[:2]
        self.mask = None if mask is None else _arr(mask, np.float32)
        self.N, self.cap = ind.shape[0], max(1, int(max_tries))
        cfg = _config(self.cap, self.N, H, W, 1, 0, 0.0, mutpb, k_sigma, min_scale_splats,
                      max_scale_splats, self.mask, boost_only, boost_beta, schedule,
                      mut_sigma_max, mut_sigma_min, seed)
        _lib.ensure_init()
        h = C.c_void_p()
        f = C.c_float()
        check(lib.ggs_sa_create(device, C.byref(cfg), self.target.ctypes.data_as(_f32p),
                                None if self.mask is None else self.mask.ctypes.data_as(_f32p),
                                ind.ctypes.data_as(_f32p), C.byref(h), C.byref(f)),
              "ggs_sa_create")
        self.h, self.init_fit, self.last_n = h, f.value, 0
        check(lib.ggs_sa_set_incremental(h, int(bool(incremental))), "ggs_sa_set_incremental")

    def stats(self) -> Dict[str, int]:
        """Neighbours proposed and splats changed (the incremental path's work)."""
        p, c = C.c_uint64(), C.c_uint64()
        check(lib.ggs_sa_stats(self.h, C.byref(p), C.byref(c)), "ggs_sa_stats")
        return {"proposed": p.value, "changed_splats": c.value}

    def propose(self, it: int, total: int, first_try: int, n: int, draws=None) -> np.ndarray:
        out = np.empty(n, np.float32)
        keep = {}
        d = None if draws is None else C.byref(_draws_struct(draws, keep, MUTATION_KEYS))
        check(lib.ggs_sa_propose(self.h, it, total, first_try, n, d, out.ctypes.data_as(_f32p)),
              "ggs_sa_propose")
        self.last_n = n
        return out

    def commit(self, j: int, update_best: bool) -> None:
        check(lib.ggs_sa_commit(self.h, j, int(bool(update_best))), "ggs_sa_commit")

    def run(self, first_it: int, temps, total: int, tries: int, width: int = 0) -> np.ndarray:
        """Iterations first_it .. first_it+len(temps)-1 of the SA loop on the device
        (ggs_sa_run): acceptance walk and state updates included, one host sync per
        batch of rounds.  Returns the [n, 2] (best, current) energy curves."""
        t = _arr(temps, np.float64)
        out = np.empty((len(t), 2), np.float64)
        check(lib.ggs_sa_run(self.h, int(first_it), len(t), int(total), int(tries),
                             t.ctypes.data_as(_f64p), int(width), out.ctypes.data_as(_f64p)),
              "ggs_sa_run")
        return out

    def loop_state(self) -> Dict[str, float]:
        """Energies and counters of the device loop after the last ``run``."""
        b, c = C.c_double(), C.c_double()
        r, e, a = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(lib.ggs_sa_loop_state(self.h, C.byref(b), C.byref(c), C.byref(r), C.byref(e),
                                    C.byref(a)), "ggs_sa_loop_state")
        return {"best_fit": b.value, "current_fit": c.value, "rounds": r.value,
                "evaluated": e.value, "accepted": a.value}

    def read(self):
        cur = np.empty((self.N, 9), np.float32)
        best = np.empty((self.N, 9), np.float32)
        nb = np.empty((max(self.last_n, 1), self.N, 9), np.float32)
        check(lib.ggs_sa_read(self.h, cur.ctypes.data_as(_f32p), best.ctypes.data_as(_f32p),
                              nb.ctypes.data_as(_f32p)), "ggs_sa_read")
        return cur, best, nb[:self.last_n]

    def close(self) -> None:
        if getattr(self, "h", None):
            lib.ggs_sa_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 — interpreter shutdown
            pass


class DeviceGA:
    """One device-resident GA population (see module docstring)."""

    def __init__(self, target, mask, init_pop, *, tour_k: int, elite_k: int, cxpb: float,
                 mutpb: float, mut_sigma_max: Dict[str, float], mut_sigma_min: Dict[str, float],
                 schedule: str, min_scale_splats: float, max_scale_splats: float,
                 k_sigma: float = 3.0, boost_only: bool = False, boost_beta: float = 1.0,
                 seed: int = 0, device: int = 0):
        pop = _arr(init_pop, np.float32)
        P, N, Cc = pop.shape
        if Cc != 9:
            raise _lib.GGSInputError("the device GA keeps [P, N, 9] genomes")
        self.target = _arr(target, np.float32)
        H, W = self.target.shape[:2]
        self.mask = None if mask is None else _arr(mask, np.float32)
        cfg = _config(P, N, H, W, tour_k, elite_k, cxpb, mutpb, k_sigma, min_scale_splats,
                      max_scale_splats, self.mask, boost_only, boost_beta, schedule,
                      mut_sigma_max, mut_sigma_min, seed)
        self.P, self.N, self.H, self.W, self.tour_k, self.cxpb = P, N, H, W, tour_k, cxpb
        _lib.ensure_init()
        h = C.c_void_p()
        check(lib.ggs_ga_create(device, C.byref(cfg), self.target.ctypes.data_as(_f32p),
                                None if self.mask is None else self.mask.ctypes.data_as(_f32p),
                                pop.ctypes.data_as(_f32p), C.byref(h)), "ggs_ga_create")
        self.h = h

    def set_comm(self, gather) -> None:
        """Shard each generation's offspring evaluation over the ranks of an
        ``ggs.RcclGather`` (one process per GPU, identical sessions on every rank;
        ggs_ga_set_comm).  ``None``: evaluate every offspring here."""
        self._comm = gather                     # keeps the communicator alive
        check(lib.ggs_ga_set_comm(self.h, None if gather is None else gather.handle), "ggs_ga_set_comm")

    def step(self, gen: int, total: int, draws: Optional[Dict[str, np.ndarray]] = None) -> None:
        """One generation; ``draws`` in ggs/ga.py layout (see draws_from_host)."""
        if draws is None:
            check(lib.ggs_ga_step(self.h, gen, total, None), "ggs_ga_step")
            return
        keep = {}
        d = _draws_struct(draws, keep)
        check(lib.ggs_ga_step(self.h, gen, total, C.byref(d)), "ggs_ga_step")

    def run(self, first_gen: int, n_gens: int, total: int) -> None:
        check(lib.ggs_ga_run(self.h, first_gen, n_gens, total), "ggs_ga_run")

    def read(self) -> Dict[str, object]:
        pop = np.empty((self.P, self.N, 9), np.float32)
        fits = np.empty(self.P, np.float32)
        best = np.empty((self.N, 9), np.float32)
        bf = C.c_double()
        n = C.c_int32()
        check(lib.ggs_ga_read(self.h, None, None, None, None, None, C.byref(n)), "ggs_ga_read")
        curves = np.empty((n.value, 3), np.float64)
        check(lib.ggs_ga_read(self.h, pop.ctypes.data_as(_f32p), fits.ctypes.data_as(_f32p),
                              best.ctypes.data_as(_f32p), C.byref(bf),
                              curves.ctypes.data_as(_f64p), C.byref(n)), "ggs_ga_read")
        return {"population": pop, "fitness": fits, "best": best, "best_fit": bf.value,
                "curves": {"best": curves[:, 0].tolist(), "mean": curves[:, 1].tolist(),
                           "median": curves[:, 2].tolist()}}

    def close(self) -> None:
        if getattr(self, "h", None):
            lib.ggs_ga_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 — interpreter shutdown
            pass


def draws_from_host(tour_idx, perm, cx, cxu_compact, mut, N: int) -> Dict[str, np.ndarray]:
    """Pack the draws ggs/ga.py's next_generation consumed into the device layout
    (crossover masks expanded to one row per pair)."""
    npairs = len(cx)
    cx_u = np.ones((npairs, N), np.float32)
    cx_u[np.asarray(cx, bool)] = np.asarray(cxu_compact, np.float32).reshape(-1, N)
    out = {"tour_idx": tour_idx, "perm": perm, "cx": np.asarray(cx, np.int32), "cx_u": cx_u}
    out.update({k: mut[k] for k in MUTATION_KEYS})
    return out


class RecordingDraws:
    """Wraps a ggs.ga draw source and keeps, per generation, the draws
    ``next_generation`` consumed — in the device layout (``draws_from_host``)."""

    def __init__(self, inner, cxpb: float):
        self.inner, self.cxpb = inner, cxpb
        self.generations = []
        self._cur = {}

    def tournament(self, P, k):
        self._cur = {"tour_idx": np.asarray(self.inner.tournament(P, k))}
        return self._cur["tour_idx"]

    def shuffle(self, P):
        self._cur["perm"] = np.asarray(self.inner.shuffle(P))
        return self._cur["perm"]

    def uniform(self, n):
        u = np.asarray(self.inner.uniform(n))
        self._cur["cx"] = u < self.cxpb
        return u

    def generation(self, cx, n_off, N, mutpb):
        cxu, mut = self.inner.generation(cx, n_off, N, mutpb)
        c = self._cur
        self.generations.append(draws_from_host(c["tour_idx"], c["perm"], c["cx"], cxu, mut, N))
        return cxu, mut


def run_device_ga(target, imp_mask, init_pop, generations: int, *, tour_k: int, elite_k: int,
                  cxpb: float, mutpb: float, mut_sigma_max, mut_sigma_min, schedule: str,
                  min_scale_splats: float, max_scale_splats: float, k_sigma: float,
                  boost_only: bool, seed: int, chunk: int, on_chunk=None, draws=None,
                  device: int = 0):
    """algorithm.py:85-155 for ``generations`` generations on one GPU.

    ``draws``: optional list of per-generation draw dicts (replay); otherwise the
    Philox stream keyed by ``seed``.  ``on_chunk(gen, ga)`` runs every ``chunk``
    generations (progress bar, video frames)."""
    ga = DeviceGA(target, imp_mask, init_pop, tour_k=tour_k, elite_k=elite_k, cxpb=cxpb,
                  mutpb=mutpb, mut_sigma_max=mut_sigma_max, mut_sigma_min=mut_sigma_min,
                  schedule=schedule, min_scale_splats=min_scale_splats,
                  max_scale_splats=max_scale_splats, k_sigma=k_sigma, boost_only=boost_only,
                  seed=seed, device=device)
    try:
        gen = 1
        try:
            while gen <= generations:
                n = min(max(1, chunk), generations - gen + 1)
                if draws is not None:
                    for g in range(gen, gen + n):
                        ga.step(g, generations, draws[g - 1])
                else:
                    ga.run(gen, n, generations)
                gen += n
                if on_chunk is not None:
                    on_chunk(gen - 1, ga)
        except KeyboardInterrupt:                                  # algorithm.py:157-158
            print("\n[Interrupted] Returning current best individual…", flush=True)
        return ga.read()
    finally:
        ga.close()
