"""Pin the oracle (oracle/ggs_oracle.py) to the REFERENCE's own outputs.

tests/golden/*.npz were produced by tests/golden/make_golden.py, which runs the
reference's encode.py / render.py (Triton kernel under TRITON_INTERPRET=1) /
fitness.py / mask.py on CPU.  The reference ships no tests or fixtures of its
own, so these are the only known-answer vectors.

Tolerance policy:
* integer bounds: exact, except where the pre-floor/ceil value is within 4 ulp of
  an integer (torch's exp differs from ours by ≤1 ulp; such flips are ~1 per
  32k splats — none occur in these fixtures);
* preprocess floats: ≤ 8 ulp; encode: ≤ 16 ulp scaled by the conditioning of
  l22 = sqrt(syy − l21²) (catastrophic cancellation for needle-thin splats);
* rendered images: ≤ 1e-5 abs here (north-star bar is 1e-4);
* fitness scalars: rel ≤ 1e-5 (the reference reduces in float32).
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest

import ggs_oracle as O
from conftest import GOLDEN, load_golden

EPS = np.finfo(np.float32).eps


def _ulp_err(a, ref):
    ref = np.asarray(ref, np.float64)
    return np.abs(np.asarray(a, np.float64) - ref) / np.maximum(
        np.spacing(np.abs(ref.astype(np.float32))).astype(np.float64), 1e-45)


def _l22_condition(G):
    g = np.asarray(G, np.float64).reshape(-1, G.shape[-1])
    sx, sy = np.exp(g[:, 2]), np.exp(g[:, 3])
    c, s = np.cos(g[:, 4]), np.sin(g[:, 4])
    sxx = sx**2 * c**2 + sy**2 * s**2
    sxy = (sx**2 - sy**2) * s * c
    syy = sx**2 * s**2 + sy**2 * c**2
    l11 = np.sqrt(np.maximum(sxx, 1e-12))
    l21 = sxy / l11
    return syy / np.maximum(syy - l21 * l21, 1e-30)


@pytest.mark.parametrize("case", ["edge", "syn"])
def test_encode_matches_reference(case):
    d = load_golden("encode.npz")
    G, ref = d[f"{case}_in"], d[f"{case}_out"]
    out = O.genome_to_renderer_batched(G)
    assert out.shape == ref.shape and out.dtype == np.float32
    np.testing.assert_array_equal(out[..., :2], ref[..., :2])
    np.testing.assert_array_equal(out[..., 5:], ref[..., 5:])          # clamp is exact
    kappa = _l22_condition(G).reshape(ref.shape[:-1])
    for col in (2, 3, 4):
        tol = 16 * EPS * (1 + np.abs(ref[..., col])) * np.maximum(kappa, 1.0)
        err = np.abs(out[..., col].astype(np.float64) - ref[..., col])
        assert (err <= tol).all(), (col, err.max(), np.argmax(err - tol))


def _pre_cases():
    d = load_golden("preprocess.npz")
    return sorted({k.split("__")[0] for k in d.files})


@pytest.mark.parametrize("case", _pre_cases())
def test_preprocess_matches_reference(case):
    d = load_golden("preprocess.npz")
    H, W, k = d[f"{case}__HWk"]
    out = O.preprocess(d[f"{case}__in"], int(H), int(W), float(k), with_prefloor=True)
    for key in O.BOUND_KEYS:
        ref = d[f"{case}__{key}"]
        bad = np.nonzero(out[key] != ref)[0]
        pre = out["prefloor"][key][bad].astype(np.float64)
        near = np.abs(pre - np.round(pre)) <= 4 * np.spacing(np.abs(pre).astype(np.float32))
        assert near.all(), (key, bad[~near])
    for key in O.FLOAT_KEYS:
        assert _ulp_err(out[key], d[f"{case}__{key}"]).max() <= 8, key


def _render_cases():
    return sorted(os.path.basename(p)[7:-4] for p in glob.glob(os.path.join(GOLDEN, "render_*.npz")))


@pytest.mark.parametrize("case", _render_cases())
def test_render_matches_reference(case):
    d = load_golden(f"render_{case}.npz")
    H, W, k = d["HWk"]
    out = O.render(d["genomes"], int(H), int(W), k_sigma=float(k), background=tuple(d["bg"]))
    imgs = [key for key in d.files if key.startswith("img_t")]
    assert imgs
    for key in imgs:
        ref = d[key].reshape(out.shape)
        np.testing.assert_allclose(out, ref, atol=1e-5, rtol=0, err_msg=key)


def test_reference_render_is_tile_invariant():
    """The SURVEY finding the tile-free oracle relies on: the reference's
    output does not depend on its tile size (16 / 32 / 64)."""
    n = 0
    for case in _render_cases():
        d = load_golden(f"render_{case}.npz")
        imgs = [d[key] for key in sorted(d.files) if key.startswith("img_t")]
        for other in imgs[1:]:
            np.testing.assert_array_equal(imgs[0], other)
            n += 1
    assert n >= 4


@pytest.mark.parametrize("case", ["f64", "f128", "f40x56"])
def test_fitness_matches_reference(case):
    d = load_golden("fitness.npz")
    H, W = (int(v) for v in d[f"{case}__HW"])
    pop, tgt, mask = d[f"{case}__pop"], d[f"{case}__target"], d[f"{case}__mask"]
    plist = list(pop)
    for mode, kw in (("none", {}), ("weighted", {"weight_mask": mask}),
                     ("boost", {"weight_mask": mask, "boost_only": True})):
        got = O.fitness_many(plist, tgt, H, W, 3.0, **kw)
        np.testing.assert_allclose(got, d[f"{case}__{mode}"], rtol=1e-5, atol=0, err_msg=mode)
    chunked = O.fitness_population(plist, tgt, H, W, 3.0, chunk=2, weight_mask=mask)
    np.testing.assert_allclose(chunked, d[f"{case}__pop_chunk2"], rtol=1e-5)


def test_weighted_with_unit_mask_is_three_times_mse():
    """Σ w·d² / Σ w with w ≡ 1 is 3× the per-element mean."""
    d = load_golden("fitness.npz")
    H, W = (int(v) for v in d["f64__HW"])
    pop, tgt = list(d["f64__pop"]), d["f64__target"]
    w1 = O.fitness_many(pop, tgt, H, W, 3.0, weight_mask=np.ones((H, W), np.float32))
    np.testing.assert_allclose(w1, 3 * O.fitness_many(pop, tgt, H, W, 3.0), rtol=1e-12)


def test_synthetic_population_ranges():
    G = O.synthetic_population(4, 256, 512, 512, seed=0)
    assert G.shape == (4, 256, 9) and G.dtype == np.float32
    assert (G[..., :2] >= 0).all() and (G[..., :2] <= 1).all()
    s = np.exp(G[..., 2:4].astype(np.float64))
    assert s.min() >= 3.0 - 1e-4 and s.max() <= 51.2 + 1e-3
    assert (G[..., 8] >= 180).all() and (G[..., 5:9] <= 255).all()


def test_oracle_window_render_equals_crop_of_full_render():
    pop = O.synthetic_population(2, 40, 100, 70, seed=3)
    G = O.genome_to_renderer_batched(pop)
    full = O.render(G, 100, 70)
    for win in ((10, 57, 3, 66), (0, 100, 0, 70), (99, 100, 69, 70)):
        y0, y1, x0, x1 = win
        np.testing.assert_array_equal(O.render(G, 100, 70, window=win), full[:, y0:y1, x0:x1])


def test_headline_config_matches_reference():
    """BASELINE.json configs[1] itself (512x512, 256 splats): the oracle's encode,
    full-canvas render and weighted / plain / boost fitness against the reference
    run on the same candidate (tests/golden/make_golden_512.py: tile-64 image,
    tile-32 fitness_many) — the headline config pinned directly, not only through
    the small fixtures above."""
    d = load_golden("headline_512.npz")
    H, W, k = (float(v) for v in d["HWk"])
    H, W = int(H), int(W)
    g9, ref9 = O.genome_to_renderer_batched(d["pop"]), d["genomes"]
    np.testing.assert_array_equal(g9[..., :2], ref9[..., :2])
    np.testing.assert_array_equal(g9[..., 5:], ref9[..., 5:])
    kappa = _l22_condition(d["pop"]).reshape(ref9.shape[:-1])       # as test_encode_matches_reference
    for col in (2, 3, 4):
        tol = 16 * EPS * (1 + np.abs(ref9[..., col])) * np.maximum(kappa, 1.0)
        assert (np.abs(g9[..., col].astype(np.float64) - ref9[..., col]) <= tol).all(), col
    img = O.render(d["genomes"], H, W, k_sigma=k)
    np.testing.assert_allclose(img, d["img_t64"], atol=1e-5, rtol=0)
    tgt = d["target_u8"].astype(np.float32) / np.float32(255.0)
    for mode, kw in (("none", {}), ("weighted", {"weight_mask": d["mask"]}),
                     ("boost", {"weight_mask": d["mask"], "boost_only": True})):
        got = O.fitness_many(list(d["pop"]), tgt, H, W, k, **kw)
        np.testing.assert_allclose(got, d[f"fit_{mode}"], rtol=1e-5, err_msg=mode)
