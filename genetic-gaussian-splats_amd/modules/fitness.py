"""Drop-in for the reference's modules/fitness.py (fitness.py:1-47).

One libggs.so call per batch: encode + prep + raster + fused weighted-L2
reduction + fixed-order float64 finalize; the candidate images never reach HBM.
``tile`` and ``device`` are accepted and ignored (results are tile-invariant).
"""
from __future__ import annotations

from typing import List

import numpy as np

from modules._compat import first, ggs, is_torch, like


def fitness_many(pop_batch, target, H: int, W: int, k_sigma: float, device, tile: int = 32,
                 weight_mask=None, boost_only: bool = False, boost_beta: float = 1.0):
    """fitness.py:7-31 → per-candidate fitness [B] (float32)."""
    G = pop_batch if not isinstance(pop_batch, (list, tuple)) else \
        np.stack([ggs.as_f32(p) for p in pop_batch], 0)
    out = ggs.fitness(G, target, H, W, k_sigma, weight_mask=weight_mask,
                      boost_only=boost_only, boost_beta=boost_beta)
    ref = first(pop_batch) if isinstance(pop_batch, (list, tuple)) else pop_batch
    return like(out, ref) if is_torch(ref) else out


def fitness_population(population, target, H: int, W: int, k_sigma: float, device,
                       tile: int = 32, chunk: int | None = None, weight_mask=None,
                       boost_only: bool = False) -> List[float]:
    """fitness.py:34-47 → List[float] (chunk bounds the per-call batch only)."""
    return ggs.fitness_population(population, target, H, W, k_sigma, chunk=chunk,
                                  weight_mask=weight_mask, boost_only=boost_only)
