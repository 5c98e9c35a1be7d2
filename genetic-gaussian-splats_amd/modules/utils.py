"""Drop-in for the reference's modules/utils.py (utils.py:1-151): genome
helpers, frame/curve outputs and the renderer prewarm, over ggs/ga.py and the
libggs renderer (numpy in → numpy out; torch in → torch out)."""
from __future__ import annotations

import math
from typing import Dict, Sequence

import numpy as np

from modules._compat import ggs, is_torch, like
from ggs import ga as _ga

build_mut_sigma = _ga.build_mut_sigma                    # utils.py:31-33
save_curves_csv = _ga.save_curves_csv                    # utils.py:133-151


def wrap_angle(theta):
    """utils.py:10-12: (θ + π) mod 2π − π (float32, Python-style modulo)."""
    return like(_ga.wrap_angle(ggs.as_f32(theta)), theta)


def _anneal_factor(gen, total, kind):
    """utils.py:15-28."""
    return _ga.anneal_factor(gen, total, kind)


def clamp_genome(ind, H: int, W: int, min_scale_splats: float, max_scale_splats: float):
    """utils.py:36-45 (in place for numpy arrays and torch tensors; returns ind)."""
    if is_torch(ind):
        out = _ga.clamp_genome(np.array(ggs.as_f32(ind), copy=True), H, W, min_scale_splats,
                               max_scale_splats)
        ind.copy_(like(out, ind))
        return ind
    return _ga.clamp_genome(ind, H, W, min_scale_splats, max_scale_splats)


def render_axes_angle_to_img(ind_axes_angle, Hsnap: int, Wsnap: int, k_sigma: float,
                             device) -> np.ndarray:
    """utils.py:48-58 → uint8 [H, W, 3]."""
    G = ggs.as_f32(ind_axes_angle)
    G = G[None] if G.ndim == 2 else G
    img = ggs.render(ggs.encode(G), Hsnap, Wsnap, k_sigma=k_sigma)[0]
    return (np.clip(img, 0, 1) * 255.0).astype("uint8")


def save_frame_png(gen: int, ind_axes_angle, pad: int, prefix: str, video_dir: str, H: int,
                   W: int, k_sigma: float, device, save_video: bool = True):
    """utils.py:61-69."""
    _ga.save_frame_png(gen, ggs.as_f32(ind_axes_angle), pad, prefix, video_dir, H, W, k_sigma,
                       device, save_video)


def prewarm_renderer(H: int, W: int, k_sigma: float, device):
    """utils.py:72-82: one tiny render twice (initialises the HIP context)."""
    dummy = np.array([[[0.5, 0.5, math.log(2.0), math.log(2.0), 0.0, 128.0, 128.0, 128.0,
                        255.0]]], np.float32)
    for _ in range(2):
        ggs.render(dummy, min(8, H), min(8, W), k_sigma=k_sigma)


def save_loss_curve_png(curves: Dict[str, Sequence[float]], out_path: str,
                        title: str = "GA fitness over generations", xlabel: str = "Generation",
                        ylabel: str = "MSE", log_y: bool = False, dpi: int = 144):
    """utils.py:85-130."""
    _ga.save_loss_curve_png(curves, out_path, title, xlabel, ylabel, log_y, dpi)
