"""Degenerate splats: the lanes the raster's row-ratio clamp protects.

The raster walks a splat's rows with a multiplicative recurrence f <- f * r,
seeded by the exact value of the visit's first row pair, whose ratio to the next
pair is r = 2^d, d = 16 Cc (qy + 4) + 8 Bc qx (csrc/ggs_kernels.hip GGS_RATIO,
csrc/ggs_prep.h make_rec).  On a lane whose seed is 0 — a column outside the
splat's AABB (px = -inf) or a conic term that is not finite — d can exceed the
float exponent range, r = inf and 0 * inf = NaN; the kernel clamps d at 100.
Round 4 found that no parity test pinned those lanes (only a configs[4] SA
trajectory moved when the clamp was removed).  These fixtures contain them, and a
CPU check restating make_rec's d proves it:

* thin rotated splats (render.py:19-21 + 32-38 with |l21| / l22 up to 8): AABBs
  wide enough to cut a strip's 16 columns, tall enough to cross a 128-row tile
  edge; only ~0.7 % of such splats have dead lanes with d > 100 in a walk
  (the seed guard sends most of them down the exact path), so those are drawn
  from a seeded pool by the same CPU restatement;
* l22 at the 1e-6 clamp of render.py:20 (syy = 1e12) with large |l21|,
  positioned so every pixel's quadratic form is >= 4e10 (f = 0 everywhere in the
  reference too: no cancellation to a negative exponent);
* non-finite conic terms: l11 = l22 = 1e-6 and l21 = 1e8 (sxx = i11^2 + i21^2 =
  inf, render.py:36) at a non-integer centre (qx != 0: the reference's quad is
  inf, f = 0);
* axes-angle genomes for the fitness modes: the thin rows in axes-angle form
  (the same covariance) and axis-aligned splats with sigma_y = 1e-7
  (encode.py:18: l22 at its 1e-6 clamp);
* alpha 255 throughout.

Bars: images <= 1e-4 abs against the oracle, fitness rel <= 1e-5 in all three
modes (fitness.py:16-31), and the folded finalize equal to the separate one.
"""
from __future__ import annotations

import functools

import numpy as np
import pytest

import ggs_oracle as O

H = W = 256
TILE, TILE_H, NPK = 64, 128, 16
K = np.float32(-0.72134752044448170)     # -0.5 log2(e), make_rec


def _thin(rng, M, y_spread=60.0):
    """M thin rotated renderer rows: l22 0.35-0.9 px, |l21| / l22 <= 8 (the
    quadratic form's terms stay below ~600 over the AABB: its float32 rounding
    moves f by < 1e-4), centres spread over the tile edge at row 128."""
    l11 = rng.uniform(4, 20, M)
    l22 = rng.uniform(0.35, 0.9, M)
    l21 = rng.uniform(-8, 8, M) * l22
    g = np.empty((M, 9), np.float32)
    g[:, 0] = rng.uniform(0.05, 0.95, M)
    g[:, 1] = (128 + rng.uniform(-y_spread, y_spread, M)) / (H - 1)
    g[:, 2], g[:, 3], g[:, 4] = np.log(l11), np.log(l22), l21
    g[:, 5:8] = rng.uniform(0, 255, (M, 3))
    g[:, 8] = 255.0
    return g


def _to_axes(g9):
    """Renderer rows -> axes-angle rows with the same covariance (float64
    eigen-decomposition); encode.py:4-59 maps them back to within float32
    rounding of the Cholesky factor."""
    l11, l22, l21 = np.exp(g9[:, 2].astype(np.float64)), np.exp(g9[:, 3].astype(np.float64)), \
        g9[:, 4].astype(np.float64)
    sxx, sxy, syy = l11 ** 2, l11 * l21, l21 ** 2 + l22 ** 2
    disc = np.sqrt((sxx - syy) ** 2 / 4 + sxy ** 2)
    out = g9.copy()
    out[:, 2] = 0.5 * np.log((sxx + syy) / 2 + disc)
    out[:, 3] = 0.5 * np.log((sxx + syy) / 2 - disc)
    out[:, 4] = 0.5 * np.arctan2(2 * sxy, sxx - syy)
    return out


def _clamp_relevant(g9, axes=False):
    """The rows of g9 that, alone in a candidate, walk a recurrence with a dead
    lane at d > 100 (after encode when `axes`)."""
    G = g9[:, None, :]
    if axes:
        G = O.genome_to_renderer_batched(G)
    n = np.array([ratio_clamp_lanes(G[i:i + 1])[0][0] for i in range(len(G))])
    return g9[n > 0]


@functools.lru_cache(maxsize=None)
def _renderer_fixture(seed=3, B=4):
    """[B, N, 9] renderer genomes (x, y, log l11, log l22, l21, r, g, b, a)."""
    rng = np.random.default_rng(seed)
    pool = _clamp_relevant(_thin(rng, 4000))          # ~0.7 % of thin splats qualify
    assert len(pool) >= 4 * B, len(pool)
    rows = []
    for b in range(B):
        g = []
        # ordinary splats under and over the degenerate ones (blending matters)
        for _ in range(24):
            g.append([rng.uniform(0.1, 0.9), rng.uniform(0.1, 0.9), np.log(rng.uniform(3, 20)),
                      np.log(rng.uniform(3, 20)), rng.uniform(-5, 5), *rng.uniform(0, 255, 3),
                      rng.uniform(180, 255)])
        # thin rotated: four that reach the clamp, 44 more
        g.extend(pool[4 * b:4 * b + 4].tolist())
        g.extend(_thin(rng, 44).tolist())
        # l22 at the 1e-6 clamp, |l21| = 5, slope l21 / l11 = 2: the centre offsets
        # (0.25, 0.3) keep qy - 2 qx at least 0.2 from 0 on every pixel
        for j in range(8):
            cx, cy = 20 + 28 * j + 0.25, 30 + 25 * j + 0.3
            g.append([cx / (W - 1), cy / (H - 1), np.log(2.5), -30.0, 5.0 * (1 if j % 2 else -1),
                      *rng.uniform(0, 255, 3), 255.0])
        # non-finite sxx: l11 = l22 = 1e-6, l21 = 1e8, centre column non-integer
        for j in range(4):
            cx = 37 + 50 * j + 0.4
            g.append([cx / (W - 1), rng.uniform(0.2, 0.8), -30.0, -30.0, 1e8 * (1 if j % 2 else -1),
                      *rng.uniform(0, 255, 3), 255.0])
        rows.append(g)
    return np.asarray(rows, np.float32)


@functools.lru_cache(maxsize=None)
def _axes_fixture(seed=5, B=6):
    """[B, N, 9] axes-angle genomes (x, y, a_log, b_log, theta, r, g, b, a)."""
    rng = np.random.default_rng(seed)
    base = O.synthetic_population(B, 24, H, W, seed=seed)
    pool = _clamp_relevant(_to_axes(_thin(rng, 5000)), axes=True)
    assert len(pool) >= 3 * B, len(pool)
    thin = np.stack([np.concatenate([pool[3 * b:3 * b + 3], _to_axes(_thin(rng, 37))]) for b in range(B)])
    flat = np.empty((B, 6, 9), np.float32)                             # l22 -> 1e-6 clamp
    flat[..., 0] = rng.uniform(0.1, 0.9, (B, 6))
    flat[..., 1] = rng.uniform(0.1, 0.9, (B, 6))
    flat[:, 0, 1] = 0.0                                                # cy = 0: one visible row
    flat[..., 2] = np.log(rng.uniform(5, 20, (B, 6)))
    flat[..., 3] = np.log(1e-7)
    flat[..., 4] = 0.0
    flat[..., 5:8] = rng.uniform(0, 255, (B, 6, 3))
    flat[..., 8] = 255.0
    return np.ascontiguousarray(np.concatenate([base, thin, flat], 1), np.float32)


def ratio_clamp_lanes(G9, H=H, W=W, k=3.0):
    """Restates make_rec's d and the raster's visit geometry (float32 numpy):
    per candidate, the number of (splat, strip, lane) visits that walk the row
    recurrence (more than one row pair in the tile, the seed guard not tripped)
    on a lane whose seed is 0 — outside the AABB's columns or a non-finite px —
    with d > 100 on the first pair, i.e. the lanes where r = 2^d would be inf
    without the clamp.  Also returns the count of splats with a non-finite
    conic term."""
    G9 = np.asarray(G9, np.float32)
    out, nonfinite = [], 0
    lane = np.arange(64)
    cols16, ph = lane & 15, lane >> 4
    with np.errstate(all="ignore"):
        for g in G9:
            p = O.preprocess(g, H, W, k)
            A = K * p["sxx"]
            Bc = np.float32(2.0) * K * p["sxy"]
            Cc = K * p["syy"]
            la = np.where(p["a"] > 0, np.log2(p["a"]), -np.inf).astype(np.float32)
            nonfinite += int((~np.isfinite(p["sxx"]) | ~np.isfinite(p["sxy"]) | ~np.isfinite(p["syy"])).sum())
            n = 0
            for i in range(len(g)):
                x0, x1, y0, y1 = (int(p[q][i]) for q in ("x0", "x1", "y0", "y1"))
                for ty0 in range(0, H, TILE_H):
                    dy0, dy1 = y0 - ty0, y1 - ty0
                    if dy1 < 0 or dy0 > TILE_H - 1:
                        continue
                    gA, gB = max(dy0, 0) >> 2, min(dy1, TILE_H - 1) >> 2
                    kA = gA >> 1
                    kB = NPK if dy1 >= TILE_H - 1 else gB >> 1
                    if kB <= kA:                                  # one pair: no recurrence
                        continue
                    for sx0 in range(0, W, 16):
                        if x1 < sx0 or x0 > sx0 + 15:
                            continue
                        col = (sx0 + cols16).astype(np.float32)
                        qx = col - p["cx"][i]
                        px = (A[i] * qx) * qx + la[i]
                        dead = (col < x0) | (col > x1) | ~(px > -np.inf)
                        qy = (np.float32(ty0 + 8 * kA) + ph.astype(np.float32)) - p["cy"][i]
                        e = qy * (Cc[i] * qy + Bc[i] * qx) + px
                        live_small = ~dead & (e < -100)           # the seed guard would trip
                        if live_small.any():
                            continue
                        d = np.float32(16.0) * Cc[i] * (qy + 4) + np.float32(8.0) * Bc[i] * qx
                        n += int((dead & ~(d <= 100)).sum())
            out.append(n)
    return np.asarray(out), nonfinite


def test_fixtures_contain_the_lanes_the_ratio_clamp_protects():
    """CPU: the render fixture has dead lanes with d > 100 in recurrence walks in
    every candidate and non-finite conic terms; so does the fitness fixture
    (after encode.py's Cholesky) — otherwise the GPU tests below prove nothing."""
    G = _renderer_fixture()
    lanes, nonfinite = ratio_clamp_lanes(G)
    assert (lanes > 100).all(), lanes
    assert nonfinite >= 4 * 4
    thin, _ = ratio_clamp_lanes(G[:, 24:72])          # the well-formed thin splats alone
    assert (thin > 0).all(), thin
    G9 = O.genome_to_renderer_batched(_axes_fixture())
    lanes, _ = ratio_clamp_lanes(G9)
    assert (lanes > 0).all(), lanes
    with np.errstate(all="ignore"):
        p = O.preprocess(G9.reshape(-1, 9), H, W)
    assert (np.exp(G9[..., 3]) <= np.float32(1e-6) * 1.0001).sum() >= 6     # l22 at its clamp
    assert (p["syy"] >= 1e11).sum() >= 6


def test_oracle_is_finite_on_the_fixtures():
    with np.errstate(all="ignore"):
        img = O.render(_renderer_fixture(), H, W)
        pop = _axes_fixture()
        fit = O.fitness_many(list(pop), np.full((H, W, 3), 0.5, np.float32), H, W, 3.0)
    assert np.isfinite(img).all() and np.isfinite(fit).all()


@pytest.mark.gpu
def test_degenerate_render_matches_oracle():
    import ggs
    G = _renderer_fixture()
    with np.errstate(all="ignore"):
        ref = O.render(G, H, W)
    got = ggs.render(G, H, W)
    assert np.isfinite(got).all()
    err = float(np.abs(got - ref).max())
    assert err <= 1e-4, err
    # the same splats alone on the white canvas: the invisible ones leave it white
    with np.errstate(all="ignore"):
        inv = ggs.render(G[:, 72:], H, W)
    assert np.array_equal(inv, np.ones_like(inv))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["none", "weighted", "boost"])
def test_degenerate_fitness_matches_oracle(mode, monkeypatch):
    import ggs
    from ggs import hip
    pop = _axes_fixture()
    rng = np.random.default_rng(11)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.4, 1.0, (H, W)).astype(np.float32)
    kw = {} if mode == "none" else {"weight_mask": mask, "boost_only": mode == "boost"}
    with np.errstate(all="ignore"):
        ref = O.fitness_many(list(pop), tgt, H, W, 3.0, **kw)
    assert np.isfinite(ref).all()
    got = ggs.fitness(pop, tgt, H, W, 3.0, **kw)
    np.testing.assert_allclose(got, ref, rtol=1e-5)
    # the folded finalize (the device GA's raster instance) gives the same bits
    fm = {"none": ggs.GGS_FIT_NONE, "weighted": ggs.GGS_FIT_WEIGHTED, "boost": ggs.GGS_FIT_BOOST}[mode]
    st = hip.Stream()
    g, t, m = (hip.DeviceArray.from_host(a) for a in (pop, tgt, mask))
    plan = ggs.TargetPlan(0, st.handle, t.ptr, m.ptr, fm, 1.0, H, W)
    outs = []
    for fold in ("0", "1"):
        monkeypatch.setenv("GGS_FITNESS_FOLD", fold)
        o = hip.DeviceArray((pop.shape[0],))
        plan.fitness_device(st.handle, g.ptr, pop.shape[0], pop.shape[1], 9, 3.0, o.ptr)
        st.synchronize()
        outs.append(o.to_host())
    plan.close()
    np.testing.assert_array_equal(outs[0], outs[1])
    np.testing.assert_array_equal(outs[0], np.asarray(got, np.float32))
