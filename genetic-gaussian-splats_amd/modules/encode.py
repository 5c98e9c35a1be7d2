"""Drop-in for the reference's modules/encode.py (encode.py:1-79), on the GPU.

Uses the same deterministic float32 exp/log/sin/cos as the fused fitness
pipeline (csrc/ggs_detmath.h), so a genome encoded here and rendered with
``render_splats_rgb_triton`` gives bit-identical splat bounds to
``fitness_population`` on the same axes-angle genome.
"""
from __future__ import annotations

import numpy as np

from modules._compat import ggs, like


def axes_angle_to_cholesky(a_log, b_log, theta):
    """encode.py:4-24 → (log l11, log l22, l21)."""
    a = ggs.as_f32(a_log)
    rows = np.zeros(a.shape + (9,), np.float32)
    rows[..., 2] = a
    rows[..., 3] = ggs.as_f32(b_log)
    rows[..., 4] = ggs.as_f32(theta)
    r = ggs.encode(rows)
    return tuple(like(np.ascontiguousarray(r[..., j]), a_log) for j in (2, 3, 4))


def genome_to_renderer(ind_axes_angle):
    """encode.py:27-59: [N,C] (or [C]) axes-angle → [N,9] renderer genome."""
    g = ggs.as_f32(ind_axes_angle)
    if g.ndim == 1:
        g = g[None]
    return like(ggs.encode(g), ind_axes_angle)


def genome_to_renderer_batched(G_axes):
    """encode.py:62-79: [B,N,C] → [B,N,9]."""
    g = ggs.as_f32(G_axes)
    if g.ndim != 3:
        raise ggs.GGSInputError(f"expected [B,N,C], got {tuple(g.shape)}")
    return like(ggs.encode(g), G_axes)
