"""Drop-in for the reference's modules/mask.py (mask.py:1-83): the importance
mask of the weighted fitness, restated in numpy (ggs/mask.py; one-shot host work,
pinned to the reference's output in tests/golden/mask.npz)."""
from __future__ import annotations

from modules._compat import ggs, like
from ggs import mask as _m


def compute_importance_mask(target_hw3, H: int, W: int, edge_scales=(1, 2, 4),
                            w_edge: float = 0.7, w_var: float = 0.3, gamma: float = 0.7,
                            floor: float = 0.15, smooth: int = 0, strength: float = 1.0):
    """mask.py:29-83 → [H, W] float32 (torch on the input's device for torch input)."""
    out = _m.compute_importance_mask(ggs.as_f32(target_hw3), H, W, edge_scales, w_edge, w_var,
                                     gamma, floor, smooth, strength)
    return like(out, target_hw3)
