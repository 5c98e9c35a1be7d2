"""CPU restatement of the reference's render + fitness hot path (numpy).

TEST INFRASTRUCTURE — THE ORACLE.  Only tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / the timed CPU baseline.  The product path
(``genetic-gaussian-splats_amd/``) never imports it and has no CPU fallback.

Pinning: tests/golden/*.npz were produced by running the reference itself
(``/root/reference/modules/{encode,render,fitness,mask}.py``, Triton kernel under
``TRITON_INTERPRET=1``) in the build container — see
``tests/golden/make_golden.py`` and ``tests/test_oracle_golden.py``.

What is restated (each function cites the reference lines it follows):

* ``genome_to_renderer_batched`` — encode.py:4-24, 27-59, 62-79
* ``preprocess``                 — render.py:8-47
* ``render``                     — render.py:121-200 (per-pixel painter's "over"
  blend) driven as render.py:203-252 does; the tile binning of render.py:50-118
  is an acceleration structure whose result is the per-pixel AABB test — the
  reference output is tile-size invariant, so this restatement
  walks each splat's integer AABB directly, in ascending splat index.
* ``fitness_many`` / ``fitness_population`` — fitness.py:7-47

Arithmetic: exp/log/sin/cos in the *bounds-critical* stages (encode, preprocess)
use ``oracle/detmath.py`` — the deterministic float32 functions the HIP prep
stage mirrors bit-for-bit (so integer bounds are bit-exact HIP↔oracle).  The
per-pixel stage uses ``np.exp`` in float32 exactly like the Triton interpreter
(the reference's own CPU execution of render.py:189-196), evaluated in the same
operation order.  Reductions are float64.
"""
from __future__ import annotations

import os
import sys
from typing import Dict, List, Optional, Sequence

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from detmath import EPS6, EPS12, exp_f32, log_f32, sincos_f32  # noqa: E402

_f32 = np.float32
BOUND_KEYS = ("x0", "x1", "y0", "y1")
FLOAT_KEYS = ("cx", "cy", "sxx", "sxy", "syy", "rc", "gc", "bc", "a")


def _as3d(G) -> np.ndarray:
    G = np.ascontiguousarray(G, dtype=np.float32)
    if G.ndim == 2:
        G = G[None]
    if G.ndim != 3:
        raise ValueError(f"genomes must be [B,N,C] or [N,C], got {G.shape}")
    return G


# ---------------------------------------------------------------------------
# encode.py
# ---------------------------------------------------------------------------
def axes_angle_to_cholesky(a_log, b_log, theta):
    """encode.py:4-24 — Σ from (σx, σy, θ), then its Cholesky factor, as logs."""
    sx = exp_f32(a_log)
    sy = exp_f32(b_log)
    s, c = sincos_f32(theta)
    sx2 = sx * sx                      # torch pow(x, 2) == x*x  (encode.py:11)
    sy2 = sy * sy
    c2 = c * c
    s2 = s * s
    sxx = sx2 * c2 + sy2 * s2          # encode.py:11
    sxy = ((sx2 - sy2) * s) * c        # encode.py:12
    syy = sx2 * s2 + sy2 * c2          # encode.py:13
    l11 = np.sqrt(np.maximum(sxx, EPS12))            # encode.py:16
    l21 = sxy / l11                                  # encode.py:17
    l22 = np.sqrt(np.maximum(syy - l21 * l21, EPS12))  # encode.py:18
    return log_f32(l11), log_f32(l22), l21.astype(np.float32)


def genome_to_renderer(ind) -> np.ndarray:
    """encode.py:27-59 — axes-angle [N,C] → renderer [N,9]."""
    ind = np.ascontiguousarray(ind, dtype=np.float32)
    if ind.ndim == 1:
        ind = ind[None]
    out = np.empty((ind.shape[0], 9), np.float32)
    out[:, 0:2] = ind[:, 0:2]
    a, b, c = axes_angle_to_cholesky(ind[:, 2], ind[:, 3], ind[:, 4])
    out[:, 2], out[:, 3], out[:, 4] = a, b, c
    out[:, 5:9] = np.clip(ind[:, 5:9], _f32(0.0), _f32(255.0))   # encode.py:50-56
    return out


def genome_to_renderer_batched(G_axes) -> np.ndarray:
    """encode.py:62-79 (C ≥ 9 always holds for fitness inputs)."""
    G = _as3d(G_axes)
    B, N, C = G.shape
    if C < 9:
        raise ValueError("expected at least 9 genome cols")
    return genome_to_renderer(G.reshape(B * N, C)).reshape(B, N, 9)


# ---------------------------------------------------------------------------
# render.py
# ---------------------------------------------------------------------------
def preprocess(genome, H: int, W: int, k_sigma: float = 3.0,
               with_prefloor: bool = False) -> Dict[str, np.ndarray]:
    """render.py:8-47 for a [N,C≥9] (or [B,N,C], flattened) renderer genome."""
    g = np.ascontiguousarray(genome, dtype=np.float32)
    g = g.reshape(-1, g.shape[-1]) if g.ndim != 1 else g[None]
    k = _f32(k_sigma)
    maxx, maxy = _f32(W - 1), _f32(H - 1)
    zero, one = _f32(0.0), _f32(1.0)
    cx = np.clip(g[:, 0], zero, one) * maxx                  # render.py:15
    cy = np.clip(g[:, 1], zero, one) * maxy                  # render.py:16
    l11 = np.maximum(exp_f32(g[:, 2]), EPS6)                 # render.py:19
    l22 = np.maximum(exp_f32(g[:, 3]), EPS6)                 # render.py:20
    l21 = g[:, 4]
    hx = np.maximum(k * np.abs(l11), one)                    # render.py:24
    hy = np.maximum(k * (np.abs(l21) + np.abs(l22)), one)    # render.py:25
    pre = {"x0": np.clip(cx - hx, zero, maxx), "x1": np.clip(cx + hx, zero, maxx),
           "y0": np.clip(cy - hy, zero, maxy), "y1": np.clip(cy + hy, zero, maxy)}
    out = {
        "cx": cx, "cy": cy,
        "x0": np.floor(pre["x0"]).astype(np.int32),          # render.py:27-30
        "x1": np.ceil(pre["x1"]).astype(np.int32),
        "y0": np.floor(pre["y0"]).astype(np.int32),
        "y1": np.ceil(pre["y1"]).astype(np.int32),
    }
    i11 = one / l11                                          # render.py:32-34
    i22 = one / l22
    i21 = (-l21) * (i11 * i22)
    out["sxx"] = i11 * i11 + i21 * i21                       # render.py:36-38
    out["sxy"] = i21 * i22
    out["syy"] = i22 * i22
    c255 = _f32(255.0)
    for key, col in (("rc", 5), ("gc", 6), ("bc", 7), ("a", 8)):   # render.py:40-43
        out[key] = np.clip(g[:, col], zero, c255) / c255
    out = {k_: np.ascontiguousarray(v) for k_, v in out.items()}
    if with_prefloor:
        out["prefloor"] = pre
    return out


def render(genomes, H: int, W: int, *, k_sigma: float = 3.0,
           background=(1.0, 1.0, 1.0), window=None) -> np.ndarray:
    """render.py:203-252 semantics → float32 [B,H,W,3] clamped to [0,1].

    Per pixel (X, Y) (integer coordinates), for every splat whose integer AABB
    contains it, in ascending splat index (render.py:106-108 key order):
    quad = sxx·qx² + 2·sxy·qx·qy + syy·qy², f = exp(-0.5·quad)·a,
    C = (1-f)·C + f·c  (render.py:189-196).

    ``window=(wy0, wy1, wx0, wx1)`` renders only rows wy0..wy1-1 and columns
    wx0..wx1-1 of the H×W image (same values as the full render there), so
    large configurations can be checked on a crop in seconds.
    """
    G = _as3d(genomes)
    B, N, C = G.shape
    if C < 9:
        raise ValueError("expected at least 9 genome cols")
    wy0, wy1, wx0, wx1 = window if window is not None else (0, H, 0, W)
    img = np.empty((B, wy1 - wy0, wx1 - wx0, 3), np.float32)
    img[:] = np.asarray(background, dtype=np.float32)
    two, mhalf, one = _f32(2.0), _f32(-0.5), _f32(1.0)
    for b in range(B):
        p = preprocess(G[b], H, W, k_sigma)
        canvas = img[b]
        for i in range(N):
            x0, x1, y0, y1 = (int(p[k_][i]) for k_ in BOUND_KEYS)
            x0, x1, y0, y1 = max(x0, wx0), min(x1, wx1 - 1), max(y0, wy0), min(y1, wy1 - 1)
            if x1 < x0 or y1 < y0:
                continue
            X = np.arange(x0, x1 + 1, dtype=np.float32)[None, :]
            Y = np.arange(y0, y1 + 1, dtype=np.float32)[:, None]
            qx = X - p["cx"][i]
            qy = Y - p["cy"][i]
            quad = (p["sxx"][i] * (qx * qx) + (two * p["sxy"][i]) * (qx * qy)) \
                + p["syy"][i] * (qy * qy)
            f = (np.exp(mhalf * quad) * p["a"][i])[..., None]
            col = np.array([p["rc"][i], p["gc"][i], p["bc"][i]], np.float32)
            win = canvas[y0 - wy0:y1 + 1 - wy0, x0 - wx0:x1 + 1 - wx0]
            win[...] = (one - f) * win + f * col
    np.clip(img, _f32(0.0), _f32(1.0), out=img)             # render.py:252
    return img


# ---------------------------------------------------------------------------
# fitness.py
# ---------------------------------------------------------------------------
def fitness_many(pop_batch: Sequence, target, H: int, W: int, k_sigma: float,
                 weight_mask=None, boost_only: bool = False,
                 boost_beta: float = 1.0) -> np.ndarray:
    """fitness.py:7-31 → float64 [B] (reductions in float64)."""
    G_axes = np.stack([np.asarray(p, np.float32) for p in pop_batch], 0)
    G9 = genome_to_renderer_batched(G_axes)
    imgs = render(G9, H, W, k_sigma=k_sigma)
    tgt = np.asarray(target, np.float32)
    dif2 = (imgs - tgt[None]) ** 2                            # fitness.py:16
    if weight_mask is None:
        return dif2.astype(np.float64).mean(axis=(1, 2, 3))   # fitness.py:18-19
    w = np.asarray(weight_mask, np.float32)[None, :, :, None]
    if boost_only:                                            # fitness.py:23-27
        wb = _f32(1.0) + _f32(boost_beta) * np.clip(w, _f32(0), _f32(1))
        num = (dif2 * wb).astype(np.float64).mean(axis=(1, 2, 3))
        den = wb.astype(np.float64).mean() + 1e-12
        return num / den
    num = (dif2 * w).astype(np.float64).sum(axis=(1, 2, 3))   # fitness.py:28-31
    den = w.astype(np.float64).sum() + 1e-12
    return num / den


def fitness_population(population: Sequence, target, H: int, W: int,
                       k_sigma: float, tile: int = 32, chunk: Optional[int] = None,
                       weight_mask=None, boost_only: bool = False) -> List[float]:
    """fitness.py:34-47 (chunking does not change values)."""
    if chunk is None or chunk >= len(population):
        return fitness_many(population, target, H, W, k_sigma, weight_mask,
                            boost_only).tolist()
    out: List[float] = []
    for i in range(0, len(population), chunk):
        out.extend(fitness_many(population[i:i + chunk], target, H, W, k_sigma,
                                weight_mask, boost_only).tolist())
    return out


def aabb_pairs(genomes, H: int, W: int, k_sigma: float = 3.0,
               encode: bool = False) -> int:
    """Number of (splat, pixel) pairs inside integer AABBs — the unit of work
    of render.py:164-196 (used for FLOP accounting in bench.py)."""
    G = _as3d(genomes)
    G9 = genome_to_renderer_batched(G) if encode else G
    p = preprocess(G9.reshape(-1, G9.shape[-1]), H, W, k_sigma)
    w = (p["x1"].astype(np.int64) - p["x0"] + 1).clip(0)
    h = (p["y1"].astype(np.int64) - p["y0"] + 1).clip(0)
    return int((w * h).sum())


# ---------------------------------------------------------------------------
# population.py — synthetic workload spec
# ---------------------------------------------------------------------------
def synthetic_population(B: int, N: int, H: int, W: int, seed: int = 0,
                         min_scale: float = 3.0, max_scale: float = 0.1) -> np.ndarray:
    """Axes-angle genomes with the population.py:20-46 value distributions
    (numpy RNG; the reference samples with torch's RNG, so values differ but
    the distributions match)."""
    rng = np.random.default_rng(seed)
    s_lo, s_hi = float(min_scale), float(max_scale) * float(max(H, W))

    def log_scales(m):   # population.py:6-15
        conc, eps = 8.0, 1e-6
        u = rng.beta(m * conc + eps, (1 - m) * conc + eps, size=(B, N, 1))
        return np.log(s_lo + u * (s_hi - s_lo))

    G = np.concatenate([
        rng.uniform(0.0, 1.0, (B, N, 2)),
        log_scales(0.4), log_scales(0.6),
        rng.uniform(-np.pi, np.pi, (B, N, 1)),
        rng.uniform(0.0, 256.0, (B, N, 3)),
        rng.uniform(180.0, 256.0, (B, N, 1)),
    ], axis=-1).astype(np.float32)
    G[..., 0:2] = np.clip(G[..., 0:2], 0.0, 1.0)
    G[..., 5:9] = np.clip(G[..., 5:9], 0.0, 255.0)
    return G
