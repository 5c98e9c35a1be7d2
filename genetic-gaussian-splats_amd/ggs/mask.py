"""Importance mask and target preparation (host side, numpy float32).

Restates modules/mask.py:1-83 (the per-pixel weight of the weighted fitness,
computed once per run at algorithm.py:42-49 / annealing.py:89-95) and the target
resize of algorithm.py:33-39 / annealing.py:19-26.  One-shot work off the timed
path, so it stays on the host; pinned against the reference's own output in
tests/golden/mask.npz (tests/test_mask.py).
"""
from __future__ import annotations

import numpy as np

_f32 = np.float32


def resize_bilinear(x: np.ndarray, H: int, W: int) -> np.ndarray:
    """F.interpolate(mode='bilinear', align_corners=False) over the last two axes
    of a [..., h, w] float32 array (torch's source-index rule, clamped at 0)."""
    x = np.asarray(x, np.float32)
    h, w = x.shape[-2:]
    if (h, w) == (H, W):
        return x.copy()

    def axis(n_in, n_out):
        scale = _f32(n_in) / _f32(n_out)
        src = (np.arange(n_out, dtype=np.float32) + _f32(0.5)) * scale - _f32(0.5)
        src = np.maximum(src, _f32(0.0))
        i0 = np.minimum(np.floor(src).astype(np.int64), n_in - 1)
        i1 = np.minimum(i0 + 1, n_in - 1)
        l1 = (src - i0.astype(np.float32)).astype(np.float32)
        return i0, i1, (_f32(1.0) - l1).astype(np.float32), l1

    y0, y1, wy0, wy1 = axis(h, H)
    x0, x1, wx0, wx1 = axis(w, W)
    # torch's order: interpolate along x within each source row, then along y
    cols = x[..., x0] * wx0 + x[..., x1] * wx1                   # [..., h, W]
    return (cols[..., y0, :] * wy0[:, None] + cols[..., y1, :] * wy1[:, None]).astype(np.float32)


def _luma(img_hw3: np.ndarray) -> np.ndarray:
    """mask.py:7-11 (the /255 rescale applies when max > 1.5)."""
    x = img_hw3
    if x.max() > 1.5:
        x = x / _f32(255.0)
    return (_f32(0.2126) * x[..., 0] + _f32(0.7152) * x[..., 1] + _f32(0.0722) * x[..., 2]).astype(np.float32)


def _conv3x3(y: np.ndarray, k: np.ndarray) -> np.ndarray:
    p = np.pad(y, 1)
    out = np.zeros_like(y)
    for dy in range(3):
        for dx in range(3):
            if k[dy, dx]:
                out += _f32(k[dy, dx]) * p[dy:dy + y.shape[0], dx:dx + y.shape[1]]
    return out


def _sobel(y: np.ndarray) -> np.ndarray:
    """mask.py:14-19: Sobel magnitude with zero padding."""
    kx = np.array([[-1, 0, 1], [-2, 0, 2], [-1, 0, 1]], np.float32)
    gx = _conv3x3(y, kx)
    gy = _conv3x3(y, kx.T.copy())
    return np.sqrt(gx * gx + gy * gy + _f32(1e-12)).astype(np.float32)


def _avg_pool(y: np.ndarray, k: int, stride: int, pad: int) -> np.ndarray:
    """F.avg_pool2d (count_include_pad=True) on a 2-D array."""
    p = np.pad(y, pad) if pad else y
    Ho = (p.shape[0] - k) // stride + 1
    Wo = (p.shape[1] - k) // stride + 1
    c = np.zeros((p.shape[0] + 1, p.shape[1] + 1), np.float64)
    c[1:, 1:] = p.astype(np.float64).cumsum(0).cumsum(1)
    r = np.arange(Ho) * stride
    q = np.arange(Wo) * stride
    s = c[r[:, None] + k, q[None, :] + k] - c[r[:, None], q[None, :] + k] \
        - c[r[:, None] + k, q[None, :]] + c[r[:, None], q[None, :]]
    return (s / (k * k)).astype(np.float32)


def _local_variance(y: np.ndarray, k: int = 9) -> np.ndarray:
    """mask.py:22-26."""
    mean = _avg_pool(y, k, 1, k // 2)
    mean2 = _avg_pool(y * y, k, 1, k // 2)
    return np.maximum(mean2 - mean * mean, _f32(0.0))


def _norm01(t: np.ndarray) -> np.ndarray:
    """mask.py:63-66 (torch.quantile 'linear')."""
    ql, qh = np.quantile(t.astype(np.float64), [0.02, 0.98])
    ql, qh = _f32(ql), _f32(qh)
    return np.clip((t - ql) / (qh - ql + _f32(1e-12)), _f32(0.0), _f32(1.0)).astype(np.float32)


def compute_importance_mask(target_hw3, H: int, W: int, edge_scales=(1, 2, 4),
                            w_edge: float = 0.7, w_var: float = 0.3, gamma: float = 0.7,
                            floor: float = 0.15, smooth: int = 0,
                            strength: float = 1.0) -> np.ndarray:
    """mask.py:29-83 → float32 [H, W] per-pixel weight."""
    x = np.asarray(target_hw3, np.float32)
    if x.max() > 1.5:
        x = x / _f32(255.0)
    x = np.moveaxis(resize_bilinear(np.moveaxis(x, -1, 0), H, W), 0, -1)
    y = _luma(x)
    edges = np.zeros_like(y)
    for s in edge_scales:
        if s > 1:
            e = resize_bilinear(_sobel(_avg_pool(y, s, s, 0)), H, W)
        else:
            e = _sobel(y)
        edges = edges + e
    var = _local_variance(y, 9)
    m = _norm01(_f32(w_edge) * _norm01(edges) + _f32(w_var) * _norm01(var))
    if smooth and smooth > 0:
        m = _norm01(_avg_pool(m, smooth, 1, smooth // 2))
    m = np.power(m, _f32(gamma)).astype(np.float32)
    m = (_f32(1.0 - floor) * m + _f32(floor)).astype(np.float32)
    if strength < 1.0:
        m = (_f32(1.0 - strength) * np.ones_like(m) + _f32(strength) * m).astype(np.float32)
    return m


def prepare_target(target_img, H: int, W: int) -> np.ndarray:
    """algorithm.py:33-39: float32, /255 when max > 1.5, bilinear resize to (H, W)."""
    t = np.asarray(target_img, np.float32)
    if t.max() > 1.5:
        t = t / _f32(255.0)
    if t.shape[0] != H or t.shape[1] != W:
        t = np.moveaxis(resize_bilinear(np.moveaxis(t, -1, 0), H, W), 0, -1)
    return np.ascontiguousarray(t, np.float32)
