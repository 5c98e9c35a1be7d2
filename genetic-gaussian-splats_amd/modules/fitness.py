"""Drop-in for the reference's modules/fitness.py (fitness.py:1-47).

One libggs.so call per batch: encode + prep + raster + fused weighted-L2
reduction + fixed-order float64 finalize; the candidate images never reach HBM.
``tile`` is accepted and ignored (results are tile-invariant); ``device``
selects the GPU as the reference's does ('cuda:k' → device k; 'cuda' / None →
the launcher's LOCAL_RANK, else 0) — host arrays never fan out over every GPU.
"""
from __future__ import annotations

from typing import List

import numpy as np

import sys

from modules._compat import f32_contig, first, ggs, hip_device_of, is_torch, like, stream_of


def fitness_many(pop_batch, target, H: int, W: int, k_sigma: float, device, tile: int = 32,
                 weight_mask=None, boost_only: bool = False, boost_beta: float = 1.0):
    """fitness.py:7-31 → per-candidate fitness [B] (float32)."""
    ref0 = first(pop_batch) if isinstance(pop_batch, (list, tuple)) else pop_batch
    dev = hip_device_of(ref0, target, weight_mask)
    if dev is not None:                   # torch tensors on the GPU: device pointers, no copies
        torch = sys.modules["torch"]
        G = f32_contig(torch.stack(list(pop_batch), 0) if isinstance(pop_batch, (list, tuple))
                       else pop_batch)
        if G.ndim == 2:
            G = G.unsqueeze(0)
        t = f32_contig(target)
        m = None if weight_mask is None else f32_contig(weight_mask)
        mode = (ggs.GGS_FIT_NONE if m is None else
                ggs.GGS_FIT_BOOST if boost_only else ggs.GGS_FIT_WEIGHTED)
        out = torch.empty(G.shape[0], dtype=torch.float32, device=G.device)
        ggs.fitness_device(dev, stream_of(dev), G.data_ptr(), G.shape[0], G.shape[1], G.shape[2],
                           t.data_ptr(), 0 if m is None else m.data_ptr(), mode, boost_beta, H, W,
                           k_sigma, out.data_ptr())
        return out
    G = pop_batch if not isinstance(pop_batch, (list, tuple)) else \
        np.stack([ggs.as_f32(p) for p in pop_batch], 0)
    out = ggs.fitness(G, target, H, W, k_sigma, weight_mask=weight_mask,
                      boost_only=boost_only, boost_beta=boost_beta, device=device)
    ref = first(pop_batch) if isinstance(pop_batch, (list, tuple)) else pop_batch
    return like(out, ref) if is_torch(ref) else out


def fitness_population(population, target, H: int, W: int, k_sigma: float, device,
                       tile: int = 32, chunk: int | None = None, weight_mask=None,
                       boost_only: bool = False) -> List[float]:
    """fitness.py:34-47 → List[float] (chunk bounds the per-call batch only)."""
    if len(population) and hip_device_of(first(population), target, weight_mask) is not None:
        step = len(population) if chunk is None else max(1, int(chunk))
        out: List[float] = []
        for i in range(0, len(population), step):
            out.extend(fitness_many(list(population[i:i + step]), target, H, W, k_sigma, device,
                                    tile, weight_mask, boost_only).tolist())
        return out
    return ggs.fitness_population(population, target, H, W, k_sigma, chunk=chunk,
                                  weight_mask=weight_mask, boost_only=boost_only, device=device)
