"""Parity of the HIP path (libggs.so via its C ABI) with the oracle and with the
reference's golden vectors.  Needs an MI355X: run with ``-m gpu``.

Bars (north_star / SURVEY.md §8c):
* encode + preprocess: BIT-EXACT against the oracle (integer bounds and floats) —
  both sides use the deterministic float32 functions of oracle/detmath.py;
* rendered images: ≤ 1e-4 abs against the reference golden images and the oracle;
* fitness scalars: rel ≤ 1e-5 against the reference golden values and the oracle;
* full-size (512²/256/B=128) through size-independent properties: fused fitness
  == fitness of the rendered images, bit-reproducible reruns, shard invariance.
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest

import ggs
import ggs_oracle as O
from conftest import GOLDEN, load_golden

pytestmark = pytest.mark.gpu
IMG_TOL = 1e-4
FIT_RTOL = 1e-5


def _render_cases():
    return sorted(os.path.basename(p)[7:-4] for p in glob.glob(os.path.join(GOLDEN, "render_*.npz")))


def test_shares_one_hip_runtime_with_torch():
    """libggs first, torch second (a fresh process): both see the GPU, because
    ggs/_lib.py binds libggs to torch's bundled HIP runtime (one runtime per
    process; two copies fight over the device)."""
    import subprocess
    import sys
    code = ("import numpy as np, ggs; t = np.zeros((8, 8, 3), np.float32); "
            "g = np.zeros((1, 1, 9), np.float32); print(ggs.fitness(g, t, 8, 8)); "
            "import torch; print(torch.zeros(1).cuda().device)")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "PYTHONPATH": os.pathsep.join(sys.path)})
    assert r.returncode == 0, r.stderr[-2000:]
    assert "cuda:0" in r.stdout


def test_device_present_and_library_native():
    n = ggs.ensure_init()
    assert n >= 1
    # the product path is libggs.so, loaded in-tree
    maps = open("/proc/self/maps").read()
    assert ggs.LIB_PATH in maps


# ---- deterministic math: bit-exact with oracle/detmath.py ---------------------------
def _detmath(fn, x, y=None):
    import ctypes as C
    fp = C.POINTER(C.c_float)
    x = np.ascontiguousarray(x, np.float32)
    y = None if y is None else np.ascontiguousarray(y, np.float32)
    out = np.empty_like(x)
    rc = ggs.lib.ggs_detmath_eval(fn, x.ctypes.data_as(fp), None if y is None else y.ctypes.data_as(fp),
                                  len(x), out.ctypes.data_as(fp))
    assert rc == 0, ggs._lib.last_error()
    return out


def _specials():
    return np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, 1e-38, 3.4e38, -87.0,
                     -87.00001, 88.72283, 88.72284, 88.7229, np.pi, -np.pi, 1e7, -1e7, 1e30],
                    np.float32)


def test_detmath_bit_exact():
    from detmath import exp_f32, log_f32, sincos_f32
    rng = np.random.default_rng(0)
    bits = rng.integers(0, 2**32, 1_000_000, dtype=np.uint64).astype(np.uint32).view(np.float32)
    ex = np.concatenate([rng.uniform(-95, 95, 1_000_000).astype(np.float32), _specials(), bits])
    with np.errstate(over="ignore"):                       # e^100 -> +inf in float32, on purpose
        lg = np.concatenate([np.exp(rng.uniform(-100, 100, 1_000_000)).astype(np.float32),
                             _specials(), np.abs(bits)])
    tr = np.concatenate([rng.uniform(-300, 300, 1_000_000).astype(np.float32), _specials(), bits])
    s, c = sincos_f32(tr)
    for name, got, ref in (("exp", _detmath(0, ex), exp_f32(ex)), ("log", _detmath(1, lg), log_f32(lg)),
                           ("sin", _detmath(2, tr), s), ("cos", _detmath(3, tr), c)):
        same = (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))
        assert same.all(), (name, tr[~same][:5] if name in ("sin", "cos") else None)
    sq = np.abs(np.concatenate([bits, rng.uniform(0, 1e6, 1_000_000).astype(np.float32)]))
    got = _detmath(4, sq)
    with np.errstate(invalid="ignore"):                    # signalling-NaN bit patterns
        ref = np.sqrt(sq)
    assert ((got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))).all()
    num, den = bits, np.roll(bits, 1)
    with np.errstate(all="ignore"):
        ref = num / den
    got = _detmath(5, num, den)
    assert ((got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))).all()


# ---- stage parity: bit-exact with the oracle ---------------------------------------
@pytest.mark.parametrize("case", ["edge", "syn"])
def test_encode_bit_exact_vs_oracle(case):
    G = load_golden("encode.npz")[f"{case}_in"]
    np.testing.assert_array_equal(ggs.encode(G), O.genome_to_renderer_batched(G))


def test_encode_bit_exact_random_large():
    rng = np.random.default_rng(0)
    G = O.synthetic_population(8, 1024, 1024, 1024, seed=3)
    G[..., 4] = rng.uniform(-50, 50, G.shape[:2])          # unwrapped angles too
    np.testing.assert_array_equal(ggs.encode(G), O.genome_to_renderer_batched(G))


def _assert_prep_equal(got, ref):
    for k in O.BOUND_KEYS + O.FLOAT_KEYS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


@pytest.mark.parametrize("case", ["edge", "syn512", "raw", "k2", "w1"])
def test_preprocess_bit_exact_vs_oracle(case):
    d = load_golden("preprocess.npz")
    H, W, k = d[f"{case}__HWk"]
    g = d[f"{case}__in"]
    _assert_prep_equal(ggs.preprocess(g, int(H), int(W), float(k)),
                       O.preprocess(g, int(H), int(W), float(k)))


def test_preprocess_of_encoded_population_bit_exact_large():
    """The fitness path's bounds: encode -> preprocess at 1024^2, 32k splats."""
    G = O.synthetic_population(32, 1024, 1024, 1024, seed=9)
    enc = ggs.encode(G).reshape(-1, 9)
    _assert_prep_equal(ggs.preprocess(enc, 1024, 1024, 3.0), O.preprocess(enc, 1024, 1024, 3.0))


# ---- render parity ---------------------------------------------------------------------
@pytest.mark.parametrize("case", _render_cases())
def test_render_matches_reference_golden(case):
    d = load_golden(f"render_{case}.npz")
    H, W, k = d["HWk"]
    out = ggs.render(d["genomes"], int(H), int(W), k_sigma=float(k), background=tuple(d["bg"]))
    for key in (key for key in d.files if key.startswith("img_t")):
        np.testing.assert_allclose(out, d[key].reshape(out.shape), atol=IMG_TOL, rtol=0,
                                   err_msg=key)
    ref = O.render(d["genomes"], int(H), int(W), k_sigma=float(k), background=tuple(d["bg"]))
    np.testing.assert_allclose(out, ref, atol=IMG_TOL, rtol=0)


@pytest.mark.parametrize("H,W,N,B,seed", [(256, 256, 64, 2, 1), (512, 512, 256, 1, 2),
                                          (200, 333, 100, 3, 3), (1, 1, 5, 2, 4),
                                          (1, 130, 20, 1, 5), (97, 1, 20, 1, 6)])
def test_render_vs_oracle_sizes(H, W, N, B, seed):
    G9 = O.genome_to_renderer_batched(O.synthetic_population(B, N, H, W, seed=seed))
    np.testing.assert_allclose(ggs.render(G9, H, W), O.render(G9, H, W), atol=IMG_TOL, rtol=0)


def test_render_list_overflow_many_overlapping_splats():
    """> LDS list capacity per tile: 1500 large splats all covering every tile."""
    rng = np.random.default_rng(11)
    N, H, W = 1500, 96, 80
    G = np.zeros((1, N, 9), np.float32)
    G[..., 0:2] = rng.uniform(0.3, 0.7, (1, N, 2))
    G[..., 2:4] = np.log(rng.uniform(30, 60, (1, N, 2)))
    G[..., 4] = rng.uniform(-5, 5, (1, N))
    G[..., 5:8] = rng.uniform(0, 255, (1, N, 3))
    G[..., 8] = rng.uniform(0, 40, (1, N))
    np.testing.assert_allclose(ggs.render(G, H, W), O.render(G, H, W), atol=IMG_TOL, rtol=0)


@pytest.mark.parametrize("H,W", [(256, 128), (250, 120)])
def test_render_saturation_cutoff_within_2pow24(H, W):
    """Deep, opaque stacks (1,024 large splats, alpha 255): every strip's
    transmittance falls below 2^-24 after a few dozen splats and the raster stops
    (SAT_MIN_SPLATS < N).  The skipped splats can move no pixel by more than
    2^-24, so the image stays as close to the oracle as the fp32 arithmetic
    itself (1e-5 here, ten times inside the 1e-4 bar).  250x120 has strips past
    the image edge, which are never cut."""
    rng = np.random.default_rng(21)
    N = 1024
    G = np.zeros((2, N, 9), np.float32)
    G[..., 0:2] = rng.uniform(0.0, 1.0, (2, N, 2))
    G[..., 2:4] = np.log(rng.uniform(40, 90, (2, N, 2)))
    G[..., 4] = rng.uniform(-0.5, 0.5, (2, N))
    G[..., 5:8] = rng.uniform(0, 255, (2, N, 3))
    G[..., 8] = 255.0
    img = ggs.render(G, H, W)
    np.testing.assert_allclose(img, O.render(G, H, W), atol=1e-5, rtol=0)


@pytest.mark.parametrize("seed", range(24))
def test_render_and_fitness_fuzz_vs_oracle(seed):
    """Seeded random shapes and populations: canvas 1..300 per side (strips and
    tiles cut by the image edge), 1..1,500 splats (past the 512-splat cut-off
    threshold and the 1,024-entry strip list), raw genome values well outside
    the reference's ranges, k_sigma 1..4, random background; images within the
    1e-4 bar, fitness within 1e-5 relative (weighted / plain / boost modes)."""
    rng = np.random.default_rng(1000 + seed)
    H, W = int(rng.integers(1, 301)), int(rng.integers(1, 301))
    B, N = int(rng.integers(1, 4)), int(rng.choice([1, 7, 64, 300, 700, 1500]))
    G = np.empty((B, N, 9), np.float32)
    G[..., 0:2] = rng.uniform(-0.2, 1.2, (B, N, 2))
    G[..., 2:4] = rng.uniform(-1.0, np.log(0.15 * max(H, W)) + 1.0, (B, N, 2))
    G[..., 4] = rng.uniform(-8, 8, (B, N))
    G[..., 5:9] = rng.uniform(-40, 300, (B, N, 4))
    k = float(rng.uniform(1.0, 4.0))
    bg = tuple(float(v) for v in rng.uniform(0, 1, 3))
    img = ggs.render(G, H, W, k_sigma=k, background=bg)
    np.testing.assert_allclose(img, O.render(G, H, W, k_sigma=k, background=bg), atol=IMG_TOL, rtol=0)
    A = np.empty((B, N, 9), np.float32)                     # axes-angle genomes for fitness
    A[..., 0:2] = rng.uniform(0, 1, (B, N, 2))
    A[..., 2:4] = rng.uniform(np.log(1.0), np.log(0.1 * max(H, W) + 2), (B, N, 2))
    A[..., 4] = rng.uniform(-np.pi, np.pi, (B, N))
    A[..., 5:9] = rng.uniform(0, 255, (B, N, 4))
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0, 1, (H, W)).astype(np.float32)
    for m, boost in ((mask, False), (None, False), (mask, True)):
        got = ggs.fitness(A, tgt, H, W, k, weight_mask=m, boost_only=boost)
        ref = O.fitness_many(list(A), tgt, H, W, k, weight_mask=m, boost_only=boost)
        np.testing.assert_allclose(got, ref, rtol=FIT_RTOL)


def test_render_edge_inputs():
    H, W = 40, 50
    assert ggs.render(np.zeros((0, 3, 9), np.float32), H, W).shape == (0, H, W, 3)
    empty = ggs.render(np.zeros((2, 0, 9), np.float32), H, W, background=(0.2, 1.5, -1.0))
    np.testing.assert_array_equal(empty, np.broadcast_to(np.float32([0.2, 1.0, 0.0]), empty.shape))
    g = O.genome_to_renderer_batched(O.synthetic_population(2, 30, H, W, seed=1))
    g12 = np.concatenate([g, np.full((2, 30, 3), 9.0, np.float32)], -1)
    np.testing.assert_array_equal(ggs.render(g12, H, W), ggs.render(g, H, W))
    np.testing.assert_array_equal(ggs.render(g[0], H, W), ggs.render(g[:1], H, W))
    np.testing.assert_allclose(ggs.render(g, H, W, k_sigma=1.5), O.render(g, H, W, k_sigma=1.5),
                               atol=IMG_TOL, rtol=0)


# ---- fitness parity ------------------------------------------------------------------------
@pytest.mark.parametrize("case", ["f64", "f128", "f40x56"])
def test_fitness_matches_reference_golden(case):
    d = load_golden("fitness.npz")
    H, W = (int(v) for v in d[f"{case}__HW"])
    pop, tgt, mask = d[f"{case}__pop"], d[f"{case}__target"], d[f"{case}__mask"]
    for mode, kw in (("none", {}), ("weighted", {"weight_mask": mask}),
                     ("boost", {"weight_mask": mask, "boost_only": True})):
        got = ggs.fitness(pop, tgt, H, W, 3.0, **kw)
        np.testing.assert_allclose(got, d[f"{case}__{mode}"], rtol=FIT_RTOL, err_msg=mode)
        np.testing.assert_allclose(got, O.fitness_many(list(pop), tgt, H, W, 3.0, **kw),
                                   rtol=FIT_RTOL, err_msg=mode)
    chunked = ggs.fitness_population(list(pop), tgt, H, W, 3.0, chunk=2, weight_mask=mask)
    np.testing.assert_allclose(chunked, d[f"{case}__pop_chunk2"], rtol=FIT_RTOL)


def test_fitness_edge_inputs():
    """fitness.py:7-47 at the edges: an empty batch, candidates without splats (the
    background alone), an all-zero weight mask (weighted: 0 / (0 + 1e-12) = 0), mask
    values outside [0, 1] (boost clamps them, fitness.py:24), a one-pixel canvas and
    one-row / one-column canvases — against the oracle in every mode."""
    rng = np.random.default_rng(77)
    H, W = 33, 47
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0, 1, (H, W)).astype(np.float32)
    modes = ({}, {"weight_mask": mask}, {"weight_mask": mask, "boost_only": True})
    assert np.asarray(ggs.fitness(np.zeros((0, 5, 9), np.float32), tgt, H, W, 3.0)).shape == (0,)
    assert list(ggs.fitness_population([], tgt, H, W, 3.0, weight_mask=mask)) == []
    none = np.zeros((2, 0, 9), np.float32)
    for kw in modes:
        np.testing.assert_allclose(ggs.fitness(none, tgt, H, W, 3.0, **kw),
                                   O.fitness_many(list(none), tgt, H, W, 3.0, **kw), rtol=FIT_RTOL)
    pop = O.synthetic_population(3, 40, H, W, seed=8)
    zero = np.zeros((H, W), np.float32)
    np.testing.assert_array_equal(ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=zero), np.zeros(3, np.float32))
    wild = rng.uniform(-2, 3, (H, W)).astype(np.float32)
    for kw in ({"weight_mask": zero, "boost_only": True}, {"weight_mask": wild, "boost_only": True}):
        np.testing.assert_allclose(ggs.fitness(pop, tgt, H, W, 3.0, **kw),
                                   O.fitness_many(list(pop), tgt, H, W, 3.0, **kw), rtol=FIT_RTOL)
    for h, w in ((1, 1), (1, 96), (96, 1)):
        t = rng.uniform(0, 1, (h, w, 3)).astype(np.float32)
        m = rng.uniform(0, 1, (h, w)).astype(np.float32)
        p = O.synthetic_population(2, 9, h, w, seed=h * 1000 + w)
        np.testing.assert_allclose(ggs.render(O.genome_to_renderer_batched(p), h, w),
                                   O.render(O.genome_to_renderer_batched(p), h, w), atol=IMG_TOL, rtol=0)
        for kw in ({}, {"weight_mask": m}, {"weight_mask": m, "boost_only": True}):
            np.testing.assert_allclose(ggs.fitness(p, t, h, w, 3.0, **kw),
                                       O.fitness_many(list(p), t, h, w, 3.0, **kw), rtol=FIT_RTOL)


def test_fitness_vs_oracle_512():
    H = W = 512
    pop = O.synthetic_population(4, 256, H, W, seed=21)
    rng = np.random.default_rng(5)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.405, 1.0, (H, W)).astype(np.float32)
    for kw in ({}, {"weight_mask": mask}, {"weight_mask": mask, "boost_only": True}):
        np.testing.assert_allclose(ggs.fitness(pop, tgt, H, W, 3.0, **kw),
                                   O.fitness_many(list(pop), tgt, H, W, 3.0, **kw), rtol=FIT_RTOL)


def test_fitness_vs_oracle_1024_config():
    """configs[2]/[3] shape: 1024^2, 1024 splats (two candidates vs the oracle) and
    the batch invariance of the full pop-512 evaluation."""
    H = W = 1024
    pop = O.synthetic_population(512, 1024, H, W, seed=31)
    rng = np.random.default_rng(6)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.405, 1.0, (H, W)).astype(np.float32)
    full = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
    idx = [0, 511]
    np.testing.assert_allclose(full[idx], O.fitness_many(list(pop[idx]), tgt, H, W, 3.0,
                                                         weight_mask=mask), rtol=FIT_RTOL)
    np.testing.assert_array_equal(full[200:264], ggs.fitness(pop[200:264], tgt, H, W, 3.0,
                                                             weight_mask=mask))


def test_headline_config_matches_reference_golden():
    """BASELINE.json configs[1] (512x512, 256 splats) pinned directly to the
    reference (tests/golden/headline_512.npz, made by make_golden_512.py running
    render.py's Triton kernel under the interpreter and fitness.py): libggs's full
    image within 1e-4 abs of the reference's tile-64 image (render.py:203-252),
    its weighted / plain / boost fitness within 1e-5 relative of fitness_many
    (fitness.py:7-31), through the host API and the planned device path the bench
    times (ggs_plan_create + fitness)."""
    d = load_golden("headline_512.npz")
    H, W = int(d["HWk"][0]), int(d["HWk"][1])
    img = ggs.render(d["genomes"], H, W, k_sigma=float(d["HWk"][2]))
    np.testing.assert_allclose(img, d["img_t64"], atol=IMG_TOL, rtol=0)
    tgt = d["target_u8"].astype(np.float32) / np.float32(255.0)
    for mode, kw in (("none", {}), ("weighted", {"weight_mask": d["mask"]}),
                     ("boost", {"weight_mask": d["mask"], "boost_only": True})):
        got = ggs.fitness(d["pop"], tgt, H, W, 3.0, **kw)
        np.testing.assert_allclose(got, d[f"fit_{mode}"], rtol=FIT_RTOL, err_msg=mode)
    from ggs import hip
    st = hip.Stream()
    g, t, m = (hip.DeviceArray.from_host(np.ascontiguousarray(a, np.float32)) for a in (d["pop"], tgt, d["mask"]))
    out = hip.DeviceArray((1,))
    plan = ggs.TargetPlan(0, st.handle, t.ptr, m.ptr, ggs.GGS_FIT_WEIGHTED, 1.0, H, W)
    plan.fitness_device(st.handle, g.ptr, 1, d["pop"].shape[1], 9, 3.0, out.ptr)
    st.synchronize()
    np.testing.assert_allclose(out.to_host(), d["fit_weighted"], rtol=FIT_RTOL)
    plan.close()


@pytest.mark.parametrize("fold", [False, True], ids=["finalize_launch", "folded_finalize"])
def test_fused_finalize_bit_stable_under_concurrent_uneven_load(fold, monkeypatch):
    """Fitness under uneven concurrent load: four or five streams with their own
    plans and workspaces, batches of 128 / 37 / 1 candidates at 512^2, 24 at
    1024^2 and 8 at 1024^2 with 640 splats (the saturation-checking instance),
    30 launches each, enqueued interleaved with no sync; every launch's fitness
    vector equals, bit for bit, the same batch evaluated alone.

    folded_finalize runs the fitness API with the finalize folded into the raster
    (GGS_FITNESS_FOLD=1, the device GA's raster_kernel<1, *, true>): the last
    strip wave of each candidate reduces partials other waves, on any XCD, stored
    write-through, after an agent-scope acquire; the second round of launches
    checks that the per-candidate counters re-arm.  finalize_launch is the
    separate finalize kernel the fitness API uses by default."""
    from ggs import hip
    rng = np.random.default_rng(77)
    jobs = []
    monkeypatch.delenv("GGS_FITNESS_FOLD", raising=False)
    for H, B, N, seed in ((512, 128, 256, 1), (512, 37, 256, 2), (512, 1, 256, 3), (1024, 24, 512, 4),
                          (1024, 8, 640, 5)):
        pop = O.synthetic_population(B, N, H, H, seed=seed)
        tgt = rng.uniform(0, 1, (H, H, 3)).astype(np.float32)
        mask = rng.uniform(0.4, 1.0, (H, H)).astype(np.float32)
        st = hip.Stream()
        g, t, m = (hip.DeviceArray.from_host(a) for a in (pop, tgt, mask))
        plan = ggs.TargetPlan(0, st.handle, t.ptr, m.ptr, ggs.GGS_FIT_WEIGHTED, 1.0, H, H)
        jobs.append(dict(H=H, B=B, N=N, st=st, g=g, t=t, m=m, plan=plan,
                         alone=ggs.fitness(pop, tgt, H, H, 3.0, weight_mask=mask)))
    if fold:
        monkeypatch.setenv("GGS_FITNESS_FOLD", "1")
    # the path under test really runs: no finalize launch when folded
    ggs.profile_reset()
    ggs.profile_enable(True)
    j0, o0 = jobs[0], hip.DeviceArray((jobs[0]["B"],))
    j0["plan"].fitness_device(j0["st"].handle, j0["g"].ptr, j0["B"], j0["N"], 9, 3.0, o0.ptr)
    j0["st"].synchronize()
    n_fin = ggs.profile_read("finalize")[1]
    n_ras = ggs.profile_read("raster")[1]
    ggs.profile_enable(False)
    ggs.profile_reset()
    assert n_ras == 1 and n_fin == (0 if fold else 1), (n_ras, n_fin)
    np.testing.assert_array_equal(o0.to_host(), j0["alone"])
    for _ in range(2):
        outs = [[hip.DeviceArray((j["B"],)) for _ in range(30)] for j in jobs]
        for i in range(30):
            for j, o in zip(jobs, outs):
                j["plan"].fitness_device(j["st"].handle, j["g"].ptr, j["B"], j["N"], 9, 3.0, o[i].ptr)
        for j in jobs:
            j["st"].synchronize()
        for j, o in zip(jobs, outs):
            for i in range(30):
                np.testing.assert_array_equal(o[i].to_host(), j["alone"], err_msg=f"H={j['H']} B={j['B']} #{i}")
    for j in jobs:
        j["plan"].close()


@pytest.mark.parametrize("N", [512, 513])
def test_ga_default_config_vs_oracle(N):
    """The reference's shipped GA run (run_ggs.py:41, config.py:5-11): 512^2 work
    size, N_SPLATS 512, POP_SIZE 32, ELITE_K 8 -> 24 offspring evaluated per
    generation.  N = 512 and 513 straddle the raster's instance switch
    (SAT_MIN_SPLATS in csrc/ggs_kernels.hip: the saturation-checking kernel runs
    from 513 splats on).  Three of the 24 fitness values vs the oracle (rel 1e-5),
    a 128x128 centre crop of one image (1e-4 abs), and the launch of 24 equal to
    the launches of its halves (batch invariance)."""
    H = W = 512
    pop = O.synthetic_population(24, N, H, W, seed=50 + N)
    rng = np.random.default_rng(N)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.405, 1.0, (H, W)).astype(np.float32)
    full = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
    idx = [0, 11, 23]
    np.testing.assert_allclose(full[idx], O.fitness_many(list(pop[idx]), tgt, H, W, 3.0, weight_mask=mask),
                               rtol=FIT_RTOL)
    np.testing.assert_array_equal(full, np.concatenate([ggs.fitness(pop[:12], tgt, H, W, 3.0, weight_mask=mask),
                                                        ggs.fitness(pop[12:], tgt, H, W, 3.0, weight_mask=mask)]))
    img = ggs.render(ggs.encode(pop[11:12]), H, W)[0]
    win = (192, 320, 192, 320)
    ref = O.render(O.genome_to_renderer_batched(pop[11:12]), H, W, window=win)[0]
    np.testing.assert_allclose(img[192:320, 192:320], ref, atol=IMG_TOL, rtol=0)


def test_render_2048_config_crops_vs_oracle():
    """configs[4] shape (run_sags.py: 2048^2, 4096 splats, one candidate): the GPU
    image on three 96x96 crops (centre, corner, edge) vs the oracle rendering just
    those windows; fused fitness == fitness of the rendered image."""
    H = W = 2048
    pop = O.synthetic_population(1, 4096, H, W, seed=41)
    img = ggs.render(ggs.encode(pop), H, W)[0]
    for wy, wx in ((976, 976), (0, 0), (1952, 700)):
        win = (wy, wy + 96, wx, wx + 96)
        ref = O.render(O.genome_to_renderer_batched(pop), H, W, window=win)[0]
        np.testing.assert_allclose(img[wy:wy + 96, wx:wx + 96], ref, atol=IMG_TOL, rtol=0,
                                   err_msg=str(win))
    rng = np.random.default_rng(8)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.405, 1.0, (H, W)).astype(np.float32)
    fused = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
    d2 = ((img.astype(np.float64) - tgt) ** 2).sum(-1)
    ref = (d2 * mask).sum() / (mask.astype(np.float64).sum() + 1e-12)
    np.testing.assert_allclose(fused[0], ref, rtol=FIT_RTOL)


# ---- full-size properties (512^2 / 256 splats / pop 128) -------------------------------------
@pytest.fixture(scope="module")
def full_size():
    H = W = 512
    pop = O.synthetic_population(128, 256, H, W, seed=0)
    rng = np.random.default_rng(1)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.405, 1.0, (H, W)).astype(np.float32)
    return pop, tgt, mask, H, W


def test_full_size_fused_fitness_equals_fitness_of_rendered_images(full_size):
    pop, tgt, mask, H, W = full_size
    fused = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
    imgs = ggs.render(ggs.encode(pop), H, W)
    d2 = ((imgs.astype(np.float64) - tgt[None]) ** 2).sum(-1)
    ref = (d2 * mask[None]).sum((1, 2)) / (mask.astype(np.float64).sum() + 1e-12)
    np.testing.assert_allclose(fused, ref, rtol=FIT_RTOL)


def test_full_size_bit_reproducible_and_shard_invariant(full_size):
    pop, tgt, mask, H, W = full_size
    a = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
    b = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
    np.testing.assert_array_equal(a, b)
    parts = np.concatenate([ggs.fitness(pop[i:i + 37], tgt, H, W, 3.0, weight_mask=mask)
                            for i in range(0, len(pop), 37)])
    np.testing.assert_array_equal(a, parts)
    one = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask, n_devices=0)   # every GPU
    np.testing.assert_array_equal(a, one)


def test_chunked_grid_ragged_last_chunk_equals_small_batches():
    """Launches whose records exceed the raster's chunk budget run in candidate
    chunks (raster_chunk: 40 MiB of records + bounds, 80 B per splat → 128
    candidates at N = 4096).  B = 300 = 128 + 128 + 44 exercises two full chunks
    and a ragged one; every candidate's fitness and image must equal those of
    batches that fit one chunk, bit for bit."""
    H = W = 128
    N, B = 4096, 300
    pop = O.synthetic_population(B, N, H, W, seed=77)
    rng = np.random.default_rng(5)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.405, 1.0, (H, W)).astype(np.float32)
    whole = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
    parts = np.concatenate([ggs.fitness(pop[i:i + 100], tgt, H, W, 3.0, weight_mask=mask)
                            for i in range(0, B, 100)])
    np.testing.assert_array_equal(whole, parts)
    enc = ggs.encode(pop)
    imgs = ggs.render(enc, H, W)
    for i in (0, 127, 128, 255, 256, 299):
        np.testing.assert_array_equal(imgs[i], ggs.render(enc[i:i + 1], H, W)[0])


def test_full_size_sample_vs_oracle(full_size):
    pop, tgt, mask, H, W = full_size
    idx = [0, 63, 127]
    got = ggs.fitness(pop[idx], tgt, H, W, 3.0, weight_mask=mask)
    np.testing.assert_allclose(got, O.fitness_many(list(pop[idx]), tgt, H, W, 3.0, weight_mask=mask),
                               rtol=FIT_RTOL)


def test_target_cache_sees_content_change(full_size):
    pop, tgt, mask, H, W = full_size
    a = ggs.fitness(pop[:4], tgt, H, W, 3.0, weight_mask=mask)
    tgt2 = tgt.copy()
    tgt2[100:200, 100:200] = 0.0
    b = ggs.fitness(pop[:4], tgt2, H, W, 3.0, weight_mask=mask)
    assert (a != b).all()
    np.testing.assert_array_equal(ggs.fitness(pop[:4], tgt, H, W, 3.0, weight_mask=mask), a)


@pytest.mark.parametrize("n", [8, 128])
def test_target_cache_speculation_in_place_and_mode_changes(full_size, n):
    """The host API evaluates against the cached target/mask while it hashes the
    caller's arrays (ggs_capi.cpp fitness_one_device_speculative): every result
    must equal a fresh evaluation of the arrays as they are at the call — after
    in-place edits of the same buffers, a mask-only change, a mode change and a
    switch to no mask (n = 128: the bench's batch, a multi-round launch)."""
    pop, tgt, mask, H, W = full_size
    P = pop[:n]
    t, m = tgt.copy(), mask.copy()

    from ggs import hip

    def fresh(t_, m_, boost_only=False):         # device-pointer API: no host-side target cache
        st = hip.Stream()
        g, td, out = hip.DeviceArray.from_host(P), hip.DeviceArray.from_host(t_), hip.DeviceArray((len(P),))
        md = hip.DeviceArray.from_host(m_) if m_ is not None else None
        mode = ggs.GGS_FIT_NONE if m_ is None else (ggs.GGS_FIT_BOOST if boost_only else ggs.GGS_FIT_WEIGHTED)
        plan = ggs.TargetPlan(0, st.handle, td.ptr, md.ptr if md is not None else 0, mode, 1.0, H, W)
        plan.fitness_device(st.handle, g.ptr, len(P), P.shape[1], 9, 3.0, out.ptr)
        st.synchronize()
        r = out.to_host()
        plan.close()
        return r

    a = ggs.fitness(P, t, H, W, 3.0, weight_mask=m)
    np.testing.assert_array_equal(ggs.fitness(P, t, H, W, 3.0, weight_mask=m), a)   # speculation hit
    t[10:300, 50:90] = 0.25                                                           # target edited in place
    b = ggs.fitness(P, t, H, W, 3.0, weight_mask=m)
    assert (a != b).all()
    np.testing.assert_array_equal(b, fresh(t, m))
    m[:, :256] = 1.0                                                                  # mask edited in place
    c = ggs.fitness(P, t, H, W, 3.0, weight_mask=m)
    assert (c != b).any()
    np.testing.assert_array_equal(c, fresh(t, m))
    d = ggs.fitness(P, t, H, W, 3.0, weight_mask=m, boost_only=True)                  # mode change
    np.testing.assert_array_equal(d, fresh(t, m, boost_only=True))
    np.testing.assert_array_equal(a, ggs.fitness(P, tgt, H, W, 3.0, weight_mask=mask))   # back again
    e = ggs.fitness(P, t, H, W, 3.0)                                                  # no mask
    np.testing.assert_array_equal(e, fresh(t, None))
    np.testing.assert_array_equal(ggs.fitness(P, t, H, W, 3.0, weight_mask=m), c)


def test_full_size_two_streams_concurrent_bit_identical(full_size):
    """bench.py's schedule: batches alternate over two HIP streams (one workspace
    each) with both in flight at once; every batch's fitness has the same bits as
    the host API's serial evaluation."""
    torch = pytest.importorskip("torch")
    pop, tgt, mask, H, W = full_size
    dev = torch.device("cuda:0")
    ref = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
    g = torch.from_numpy(pop).to(dev)
    t_d, m_d = torch.from_numpy(tgt).to(dev), torch.from_numpy(mask).to(dev)
    sts = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    plan = ggs.TargetPlan(0, sts[0].cuda_stream, t_d.data_ptr(), m_d.data_ptr(), ggs.GGS_FIT_WEIGHTED, 1.0,
                          H, W)
    torch.cuda.synchronize(dev)
    outs = [torch.empty(len(pop), device=dev) for _ in range(8)]
    for i, o in enumerate(outs):
        plan.fitness_device(sts[i % 2].cuda_stream, g.data_ptr(), len(pop), pop.shape[1], 9, 3.0, o.data_ptr())
    torch.cuda.synchronize(dev)
    for o in outs:
        np.testing.assert_array_equal(o.cpu().numpy(), ref)


# ---- device-pointer API (inputs resident in HBM) ---------------------------------------------
def test_device_api_matches_host_api(full_size):
    torch = pytest.importorskip("torch")
    pop, tgt, mask, H, W = full_size
    dev = torch.device("cuda:0")
    dg = torch.from_numpy(pop[:16]).to(dev)
    dt = torch.from_numpy(tgt).to(dev)
    dm = torch.from_numpy(mask).to(dev)
    out = torch.empty(16, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for mode, m in ((ggs.GGS_FIT_NONE, 0), (ggs.GGS_FIT_WEIGHTED, dm.data_ptr()),
                    (ggs.GGS_FIT_BOOST, dm.data_ptr())):
        ggs.fitness_device(0, st, dg.data_ptr(), 16, 256, 9, dt.data_ptr(), m, mode, 1.0, H, W, 3.0,
                           out.data_ptr())
        torch.cuda.synchronize()
        kw = {} if mode == ggs.GGS_FIT_NONE else {"weight_mask": mask,
                                                  "boost_only": mode == ggs.GGS_FIT_BOOST}
        ref = ggs.fitness(pop[:16], tgt, H, W, 3.0, **kw)
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
        # target plan built once, reused across calls: same bits
        plan = ggs.TargetPlan(0, st, dt.data_ptr(), m, mode, 1.0, H, W)
        for _ in range(2):
            out.zero_()
            plan.fitness_device(st, dg.data_ptr(), 16, 256, 9, 3.0, out.data_ptr())
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy(), ref)
        plan.close()
    img = torch.empty((2, H, W, 3), dtype=torch.float32, device=dev)
    g9 = torch.from_numpy(ggs.encode(pop[:2])).to(dev)
    ggs.render_device(0, st, g9.data_ptr(), 2, 256, 9, H, W, 3.0, img.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(img.cpu().numpy(), ggs.render(ggs.encode(pop[:2]), H, W))


# ---- drop-in modules -------------------------------------------------------------------------
def test_drop_in_modules_numpy_and_torch():
    torch = pytest.importorskip("torch")
    from modules.fitness import fitness_many, fitness_population
    from modules.render import render_splats_rgb_triton
    from modules.encode import genome_to_renderer_batched
    d = load_golden("fitness.npz")
    H, W = (int(v) for v in d["f64__HW"])
    pop, tgt, mask = d["f64__pop"], d["f64__target"], d["f64__mask"]
    ref = d["f64__weighted"]
    got = fitness_population(list(pop), tgt, H, W, 3.0, "cuda", tile=32, chunk=None,
                             weight_mask=mask, boost_only=False)
    assert isinstance(got, list) and len(got) == len(pop)
    np.testing.assert_allclose(got, ref, rtol=FIT_RTOL)
    tp = [torch.from_numpy(p).cuda() for p in pop]
    tf = fitness_many(tp, torch.from_numpy(tgt).cuda(), H, W, 3.0, "cuda",
                      weight_mask=torch.from_numpy(mask).cuda())
    assert isinstance(tf, torch.Tensor) and tf.device.type == "cuda"
    np.testing.assert_allclose(tf.cpu().numpy(), ref, rtol=FIT_RTOL)
    g9 = genome_to_renderer_batched(torch.from_numpy(pop).cuda())
    img = render_splats_rgb_triton(g9, H, W, k_sigma=3.0, device="cuda", tile=32)
    assert isinstance(img, torch.Tensor) and img.shape == (len(pop), H, W, 3)
    with pytest.raises(AssertionError):
        render_splats_rgb_triton(g9, H, W, device="cpu")
    # the torch-on-GPU path (device pointers, no host copies) gives the host path's bits
    g9h = genome_to_renderer_batched(pop)
    np.testing.assert_array_equal(img.cpu().numpy(), render_splats_rgb_triton(g9h, H, W))
    one = render_splats_rgb_triton(g9[1].double().t().contiguous().t(), H, W)   # 2-D, f64, strided
    np.testing.assert_array_equal(one[0].cpu().numpy(), render_splats_rgb_triton(g9h[1], H, W)[0])
    for kw in ({}, {"weight_mask": mask}, {"weight_mask": mask, "boost_only": True}):
        host = fitness_many(list(pop), tgt, H, W, 3.0, "cuda", **kw)
        kwt = {k: (torch.from_numpy(v).cuda() if isinstance(v, np.ndarray) else v) for k, v in kw.items()}
        dev = fitness_many(tp, torch.from_numpy(tgt).cuda(), H, W, 3.0, "cuda", **kwt)
        np.testing.assert_array_equal(dev.cpu().numpy(), host)
        lst = fitness_population(tp, torch.from_numpy(tgt).cuda(), H, W, 3.0, "cuda", chunk=3, **kwt)
        assert lst == host.tolist()


# ---- GA layer on the GPU evaluator (§8f next #1) ----------------------------------------------
def test_ga_reference_populations_fitness_on_gpu():
    """Every population the reference's genetic_approx evaluated (recorded in
    tests/golden/ga_loop.npz) gets the same fitness from libggs (rel 1e-5), with
    the target prep and importance mask computed by ggs.mask."""
    from ggs.mask import compute_importance_mask, prepare_target
    d = load_golden("ga_loop.npz")
    H, W = int(d["cfg"][0]), int(d["cfg"][1])
    t = prepare_target(d["target"], H, W)
    m = compute_importance_mask(t, H, W, smooth=3, strength=0.7)
    for i in range(int(d["n_calls"])):
        got = ggs.fitness(d[f"call{i}__pop"], t, H, W, 3.0, weight_mask=m)
        np.testing.assert_allclose(got, d[f"call{i}__fit"], rtol=FIT_RTOL, err_msg=f"call {i}")


def test_ga_end_to_end_on_gpu():
    from modules.algorithm import genetic_approx
    from ggs import ga
    H = W = 64
    target = np.random.default_rng(4).uniform(0, 255, (80, 72, 3)).astype(np.float32)
    cfg = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0,
                              "alpha": 25.0},
               mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0,
                              "alpha": 2.0}, schedule="cosine")
    best, best_fit, st = ga.genetic_approx(
        target, H, W, "cuda", pop_size=32, n_splats=48, generations=20, tour_k=2, elite_k=8,
        cxpb=0.05, mutpb=0.05, min_scale_splats=3.0, max_scale_splats=0.1, k_sigma=3.0,
        mask_strength=0.7, boost_only=False, seed=1, progress=False, return_state=True, **cfg)
    c = st["curves"]["best"]
    assert all(b <= a for a, b in zip(c, c[1:])) and c[-1] < c[0]
    from ggs.mask import compute_importance_mask, prepare_target
    t = prepare_target(target, H, W)
    m = compute_importance_mask(t, H, W, smooth=3, strength=0.7)
    assert float(ggs.fitness(best[None], t, H, W, 3.0, weight_mask=m)[0]) == best_fit
    b2, f2 = genetic_approx(target, H, W, "cuda", 8, 16, 2, 2, 2, 0.05, 0.05, cfg["mut_sigma_max"],
                            cfg["mut_sigma_min"], "cosine", 3.0, 0.1, 3.0, 0.7, False, seed=3,
                            progress=False)
    assert b2.shape == (16, 9) and np.isfinite(f2)
