"""Drop-in for the reference's modules/population.py (population.py:1-59), in
numpy (ggs/ga.py: same distributions; the module RNG replaces torch's global
generator — reseed it with ``seed(s)``)."""
from __future__ import annotations

from typing import List

import numpy as np

from modules._compat import ggs  # noqa: F401  (locates the ggs package)
from ggs import ga as _ga

_rng_state = [None]       # made at first use from Python's `random` (ggs.ga.resolve_seed)


def _rng() -> np.random.Generator:
    if _rng_state[0] is None:
        _rng_state[0] = np.random.default_rng(_ga.resolve_seed())
    return _rng_state[0]


def seed(s) -> None:
    """Reseed the module RNG (the reference seeds torch's global RNG).  Unseeded,
    it derives its seed from Python's ``random`` at first use, so run_ggs.py's
    ``random.seed(SEED)`` (run_ggs.py:25-28) makes a run repeatable."""
    _rng_state[0] = np.random.default_rng(s)


def sample_log_scales_beta_linear(B, N, s_lo, s_hi, m=0.5, concentration=8.0, device='cuda',
                                  dtype=np.float32):
    """population.py:6-15: log(s_lo + u·(s_hi − s_lo)), u ~ Beta(m·c+ε, (1−m)·c+ε)."""
    eps = 1e-6
    u = _rng().beta(m * max(concentration, eps) + eps, (1 - m) * max(concentration, eps) + eps,
                  (B, N, 1)).astype(np.float32)
    return np.log((np.float32(s_lo) + u * np.float32(s_hi - s_lo)).astype(np.float32))


def new_population(batch_size: int, n_splats: int, H: int, W: int, min_scale_splats: float,
                   max_scale_splats: float, device='cuda', dtype=np.float32) -> np.ndarray:
    """population.py:19-46 → [B, N, 9] float32."""
    return _ga.new_population(batch_size, n_splats, H, W, min_scale_splats, max_scale_splats, _rng())


def new_individual(n_splats: int, H: int, W: int, min_scale_splats: float,
                   max_scale_splats: float, device='cuda') -> np.ndarray:
    """population.py:49-51."""
    return new_population(1, n_splats, H, W, min_scale_splats, max_scale_splats, device)[0]


def duplicate_individual(ind):
    """population.py:54-55."""
    return ind.clone() if hasattr(ind, "clone") else np.array(ind, copy=True)


def population_to_list(pop_tensor) -> List:
    """population.py:58-59."""
    return [pop_tensor[i] for i in range(pop_tensor.shape[0])]
