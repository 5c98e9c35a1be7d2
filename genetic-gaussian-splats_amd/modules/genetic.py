"""Drop-in for the reference's modules/genetic.py (genetic.py:1-93): the
per-individual operators, as thin wrappers over ggs/ga.py's batched ones (which
are replay-verified against these very functions in tests/test_ga.py).  Draws
come from a module numpy RNG (reseed with ``seed(s)``)."""
from __future__ import annotations

from typing import List

import numpy as np

from modules._compat import ggs, is_torch, like
from ggs import ga as _ga

_draws = _ga.NumpyDraws()


def seed(s) -> None:
    """Reseed the module draws (the reference uses torch's / Python's global RNGs)."""
    global _draws
    _draws = _ga.NumpyDraws(s)


def tournament_selection(pop: List, fits: List[float], k: int = 2):
    """genetic.py:8-14: best of k uniform draws (first minimum wins); a copy."""
    idx = _draws.tournament(len(pop), k)[:1]
    w = int(_ga.tournament(np.asarray(fits, np.float64), idx)[0])
    x = pop[w]
    return x.clone() if hasattr(x, "clone") else np.array(x, copy=True)


def crossover_uniform(a, b, p: float = 0.5):
    """genetic.py:17-21: per-splat (row) uniform crossover."""
    A, B = ggs.as_f32(a), ggs.as_f32(b)
    u = _draws.crossover_masks(1, A.shape[0])
    c1, c2 = _ga.crossover(A[None], B[None], u, p)
    return like(np.ascontiguousarray(c1[0]), a), like(np.ascontiguousarray(c2[0]), a)


def _ensure_one_true(mask):
    """genetic.py:24-29: if no flag is set, set one uniformly chosen flag."""
    m = np.asarray(mask, bool)
    if not m.any():
        flat = m.reshape(-1)
        flat[int(_draws.rng.integers(0, flat.size))] = True
    return m


def mutate_individual(ind, is_elite: bool, gen: int, total_gens: int, schedule: str,
                      mut_sigma_max: dict, mut_sigma_min: dict, mutpb: float, H: int, W: int,
                      min_scale_splats: float, max_scale_splats: float):
    """genetic.py:32-93 (is_elite is unused there too)."""
    G = np.array(ggs.as_f32(ind), np.float32, copy=True)[None]
    d = _draws.mutation(1, G.shape[1], mutpb)
    out = _ga.mutate_batch(G, d, gen, total_gens, schedule, mut_sigma_max, mut_sigma_min, mutpb,
                           H, W, min_scale_splats, max_scale_splats)[0]
    if is_torch(ind):
        ind.copy_(like(out, ind))          # the reference mutates in place and returns it
        return ind
    return out
