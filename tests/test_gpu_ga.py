"""The device-resident GA (ggs/ga_device.py, csrc/ggs_ga.hip) on an MI355X.

Bars:
* fed the SAME draws as the host GA (ggs/ga.py, itself replay-verified against
  the reference in tests/test_ga.py), every generation's population, fitness
  vector, best individual and curves are IDENTICAL (bit-exact);
* fed the reference's own recorded draws (tests/golden/ga_loop.npz), the
  offspring and elites are the reference's genomes bit for bit and the fitness
  values within the evaluator bar (rel 1e-5);
* with the in-kernel Philox draws: operators keep genomes in range, curves are
  monotone, the best fitness is what the evaluator returns for the best genome,
  runs are reproducible per seed.
"""
from __future__ import annotations

import numpy as np
import pytest

import ggs
from conftest import load_golden
from ggs import ga
from ggs.ga_device import DeviceGA, RecordingDraws
from ggs.mask import compute_importance_mask, prepare_target

pytestmark = pytest.mark.gpu
CFG = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0,
                          "alpha": 25.0},
           mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0,
                          "alpha": 2.0},
           schedule="cosine")          # reference modules/config.py:22-43
MIN_S, MAX_S = 3.0, 0.1


def _problem(H, W, seed):
    target = np.random.default_rng(seed).uniform(0, 255, (H + 9, W + 5, 3)).astype(np.float32)
    t = prepare_target(target, H, W)
    return target, t, compute_importance_mask(t, H, W, smooth=3, strength=0.7)


@pytest.mark.parametrize("H,W,P,N,G,tour_k,elite_k,cxpb,mutpb,boost,seed", [
    (40, 40, 17, 33, 4, 3, 4, 0.5, 0.2, False, 1),     # odd P (last pair yields one child)
    (64, 48, 32, 300, 3, 2, 8, 0.9, 0.05, True, 2),    # 256 < N <= 512: 512-thread breed workgroups
    (64, 64, 32, 512, 3, 2, 8, 0.05, 0.05, False, 6),  # config.py's shape: N 512, pop 32, elite 8
    (40, 40, 12, 700, 2, 2, 2, 0.5, 0.1, False, 7),    # 512 < N <= 1024: 1024-thread workgroups
    (32, 40, 10, 1100, 2, 2, 2, 0.5, 0.1, True, 8),    # N > 1024: generic multi-pass workgroup loops
    (24, 24, 64, 1100, 2, 2, 4, 0.5, 0.1, False, 9),   # N > 1024, P >= 64: 256-thread generic breed
    (32, 32, 8, 2, 5, 2, 1, 0.3, 0.01, False, 3),      # N = 2, rare mutation -> fallbacks
    (24, 24, 6, 1, 3, 2, 0, 0.5, 0.5, False, 4),       # N = 1: no swap; elite_k 0 -> 1
    (16, 16, 600, 3, 2, 3, 25, 0.5, 0.1, False, 5),    # P > 512: bitonic survivors path
    (24, 24, 8, 20, 3, 2, 8, 0.5, 0.2, False, 10),     # elite_k == P: no offspring survive (algorithm.py:140)
    (24, 24, 10, 40, 3, 1, 2, 0.5, 0.2, True, 11),     # tour_k 1: the tournament is one random pick
    (24, 24, 12, 30, 2, 40, 2, 0.5, 0.2, False, 12),   # 2 tour_k > 64: the per-candidate tournament loop
])
@pytest.mark.parametrize("chunk", [2, 8])   # 8 >= G: one run, every later generation a fused breed
def test_device_ga_matches_host_ga_with_same_draws(H, W, P, N, G, tour_k, elite_k, cxpb, mutpb,
                                                    boost, seed, chunk):
    target, t, m = _problem(H, W, seed)
    init = ga.new_population(P, N, H, W, MIN_S, MAX_S, np.random.default_rng(seed))
    rec = RecordingDraws(ga.NumpyDraws(seed), cxpb)
    kw = dict(pop_size=P, n_splats=N, generations=G, tour_k=tour_k, elite_k=elite_k, cxpb=cxpb,
              mutpb=mutpb, min_scale_splats=MIN_S, max_scale_splats=MAX_S, k_sigma=3.0,
              mask_strength=0.7, boost_only=boost, init_population=init, progress=False,
              return_state=True, **CFG)
    hb, hf, hs = ga.genetic_approx(target, H, W, "cuda", draws=rec, **kw)
    assert len(rec.generations) == G
    db, df, ds = ga.genetic_approx(target, H, W, "cuda", draws=rec, backend="device", chunk=chunk, **kw)
    np.testing.assert_array_equal(ds["population"], hs["population"])
    np.testing.assert_array_equal(ds["fitness"], hs["fitness"])
    np.testing.assert_array_equal(db, hb)
    assert df == hf
    for key in ("best", "mean", "median"):
        assert ds["curves"][key] == hs["curves"][key], key


def test_device_ga_replays_reference_draws():
    """Draws recorded from the reference's genetic_approx → the reference's genomes."""
    from test_ga import ReplayDraws
    d = load_golden("ga_loop.npz")
    H, W, P, N, G, tour_k, elite_k, cxpb, mutpb = d["cfg"]
    H, W, P, N, G, tour_k, elite_k = (int(v) for v in (H, W, P, N, G, tour_k, elite_k))
    # collect the per-generation draws by running the host GA on the reference's fitness
    calls = []

    def evaluate(pop):
        k = len(calls)
        ref_call = 0 if k == 0 else 2 * k - 1
        calls.append(ref_call)
        return d[f"call{ref_call}__fit"][:len(pop)].astype(np.float32)   # survivors only

    rec = RecordingDraws(ReplayDraws(d), float(cxpb))
    ga.genetic_approx(d["target"], H, W, "cuda", pop_size=P, n_splats=N, generations=G,
                      tour_k=tour_k, elite_k=elite_k, cxpb=float(cxpb), mutpb=float(mutpb),
                      min_scale_splats=MIN_S, max_scale_splats=MAX_S, k_sigma=3.0,
                      mask_strength=0.7, boost_only=False, draws=rec, evaluate=evaluate,
                      init_population=d["init"], progress=False, **CFG)
    t = prepare_target(d["target"], H, W)
    m = compute_importance_mask(t, H, W, smooth=3, strength=0.7)
    dga = DeviceGA(t, m, d["init"], tour_k=tour_k, elite_k=elite_k, cxpb=float(cxpb),
                   mutpb=float(mutpb), min_scale_splats=MIN_S, max_scale_splats=MAX_S, **CFG)
    try:
        E = max(1, elite_k)
        for g in range(1, G + 1):
            dga.step(g, G, rec.generations[g - 1])
            st = dga.read()
            off = d[f"call{2 * g - 1}__pop"]                 # the reference's offspring
            np.testing.assert_array_equal(st["population"][E:], off[:P - E], err_msg=f"gen {g}")
            np.testing.assert_allclose(st["fitness"][E:], d[f"call{2 * g - 1}__fit"][:P - E],
                                       rtol=1e-5)
            np.testing.assert_array_equal(st["population"][:E], d[f"call{2 * g}__pop"])
        np.testing.assert_array_equal(st["best"], d["best"])
        assert st["best_fit"] == pytest.approx(float(d["best_fit"]), rel=1e-5)
        np.testing.assert_allclose(st["curves"]["best"], d["curve__best"], rtol=1e-5)
        np.testing.assert_allclose(st["curves"]["mean"], d["curve__mean"], rtol=1e-5)
        np.testing.assert_allclose(st["curves"]["median"], d["curve__median"], rtol=1e-5)
    finally:
        dga.close()


def test_device_ga_philox_run():
    H = W = 64
    P, N, G = 48, 64, 30
    target, t, m = _problem(H, W, 7)
    kw = dict(pop_size=P, n_splats=N, generations=G, tour_k=3, elite_k=4, cxpb=0.3, mutpb=0.1,
              min_scale_splats=MIN_S, max_scale_splats=MAX_S, k_sigma=3.0, mask_strength=0.7,
              boost_only=False, progress=False, return_state=True, backend="device", **CFG)
    b1, f1, s1 = ga.genetic_approx(target, H, W, "cuda", seed=11, chunk=7, **kw)
    c = s1["curves"]["best"]
    assert len(c) == G + 1 and all(y <= x for x, y in zip(c, c[1:])) and c[-1] < c[0]
    assert float(ggs.fitness(b1[None], t, H, W, 3.0, weight_mask=m)[0]) == f1 == c[-1]
    np.testing.assert_array_equal(ggs.fitness(s1["population"], t, H, W, 3.0, weight_mask=m),
                                  s1["fitness"])
    Pp = s1["population"]
    assert (Pp[..., 0:2] >= 0).all() and (Pp[..., 0:2] <= 1).all()
    lo, hi = ga.scale_log_bounds(H, W, MIN_S, MAX_S)
    assert (Pp[..., 2:4] >= lo).all() and (Pp[..., 2:4] <= hi).all()
    assert (Pp[..., 4] >= -np.pi - 1e-6).all() and (Pp[..., 4] < np.pi + 1e-6).all()
    assert (Pp[..., 5:9] >= 0).all() and (Pp[..., 5:9] <= 255).all()
    # reproducible per seed and chunking-independent; another seed differs
    b2, f2, s2 = ga.genetic_approx(target, H, W, "cuda", seed=11, chunk=30, **kw)
    np.testing.assert_array_equal(s2["population"], s1["population"])
    assert f2 == f1
    _, _, s3 = ga.genetic_approx(target, H, W, "cuda", seed=12, chunk=30, **kw)
    assert not np.array_equal(s3["population"], s1["population"])


_FUSED_SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from ggs import ga
from ggs.ga_device import DeviceGA
from ggs.mask import compute_importance_mask, prepare_target
H = W = 512
P, N = int(sys.argv[3]), int(sys.argv[4])
target = np.random.default_rng(0).uniform(0, 255, (H, W, 3)).astype(np.float32)
t = prepare_target(target, H, W)
m = compute_importance_mask(t, H, W, smooth=3, strength=0.7)
init = ga.new_population(P, N, H, W, 3.0, 0.1, np.random.default_rng(0))
cfg = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0, "alpha": 25.0},
           mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0, "alpha": 2.0},
           schedule="cosine")
dga = DeviceGA(t, m, init, tour_k=2, elite_k=8, cxpb=0.05, mutpb=0.05, min_scale_splats=3.0,
               max_scale_splats=0.1, seed=1, **cfg)
dga.run(1, 25, 25)
st = dga.read()
np.savez(sys.argv[2], population=st["population"], fitness=st["fitness"], best=st["best"],
         best_fit=st["best_fit"], **{"c_" + k: np.asarray(v) for k, v in st["curves"].items()})
"""


@pytest.mark.parametrize("P,N", [(128, 256), (32, 512), (32, 1100)])
def test_device_ga_fused_breed_equals_unfused(tmp_path, P, N):
    """The fused breed (survivors + gather inside the variation kernel) against the
    five-launch generation (GGS_GA_UNFUSED=1), and the finalize folded into the
    raster against its own launch (GGS_UNFUSED_FINALIZE=1), at the bench workload
    and at the reference's shipped run (config.py: 512 splats, pop 32), 25
    generations of Philox draws in one run: identical populations, fitness, best
    and curves (N = 1100: the generic breed path, several splats per thread)."""
    import os
    import subprocess
    import sys
    pkg = os.path.dirname(os.path.dirname(ggs.__file__))
    out = {}
    for tag, env in (("fused", {}), ("unfused", {"GGS_GA_UNFUSED": "1"}),
                     ("unfused_fin", {"GGS_UNFUSED_FINALIZE": "1"})):
        path = str(tmp_path / f"{tag}.npz")
        subprocess.run([sys.executable, "-c", _FUSED_SCRIPT, pkg, path, str(P), str(N)], check=True, timeout=300,
                       env=dict(os.environ, **env))
        out[tag] = np.load(path)
    for k in out["fused"].files:
        np.testing.assert_array_equal(out["fused"][k], out["unfused"][k], err_msg=k)
        np.testing.assert_array_equal(out["fused"][k], out["unfused_fin"][k], err_msg=k)


def test_device_ga_sessions_concurrent_uneven_load_equal_solo():
    """Three device GA sessions of different shapes (each its own stream, its own
    finalize counters) stepping at the same time from three threads — the raster's
    folded finalize hands partials between waves on any XCD under uneven load —
    end in exactly the state each reaches alone."""
    import threading
    shapes = [(512, 256, 128, 1), (512, 512, 32, 2), (1024, 1024, 8, 3)]

    def run(H, N, P, seed):
        target, t, m = _problem(H, H, seed)
        init = ga.new_population(P, N, H, H, MIN_S, MAX_S, np.random.default_rng(seed))
        dga = DeviceGA(t, m, init, tour_k=2, elite_k=min(8, P - 1), cxpb=0.05, mutpb=0.05,
                       min_scale_splats=MIN_S, max_scale_splats=MAX_S, seed=seed, **CFG)
        dga.run(1, 40, 40)
        st = dga.read()
        dga.close()
        return st

    solo = [run(*sh) for sh in shapes]
    got = [None] * len(shapes)

    def worker(i):
        got[i] = run(*shapes[i])
    th = [threading.Thread(target=worker, args=(i,)) for i in range(len(shapes))]
    for x in th:
        x.start()
    for x in th:
        x.join(300)
    for a, b in zip(got, solo):
        np.testing.assert_array_equal(a["population"], b["population"])
        np.testing.assert_array_equal(a["fitness"], b["fitness"])
        assert a["best_fit"] == b["best_fit"]


def test_device_ga_read_is_idempotent_and_resumable():
    """ggs_ga_read applies a pending generation's survivors once: reading twice
    returns the same state and curve count, and stepping on after a read gives the
    same run as never reading (fused breeds across the read boundary)."""
    H = W = 48
    P, N = 24, 40
    _, t, m = _problem(H, W, 3)
    init = ga.new_population(P, N, H, W, MIN_S, MAX_S, np.random.default_rng(3))
    kw = dict(tour_k=2, elite_k=3, cxpb=0.4, mutpb=0.1, min_scale_splats=MIN_S, max_scale_splats=MAX_S,
              seed=5, **CFG)
    a, b = DeviceGA(t, m, init, **kw), DeviceGA(t, m, init, **kw)
    try:
        a.run(1, 6, 12)
        r1, r2 = a.read(), a.read()
        np.testing.assert_array_equal(r1["population"], r2["population"])
        assert r1["curves"] == r2["curves"] and len(r1["curves"]["best"]) == 7
        a.run(7, 6, 12)
        b.run(1, 12, 12)
        ra, rb = a.read(), b.read()
        for k in ("population", "fitness", "best"):
            np.testing.assert_array_equal(ra[k], rb[k], err_msg=k)
        assert ra["best_fit"] == rb["best_fit"] and ra["curves"] == rb["curves"]
    finally:
        a.close()
        b.close()


def test_device_ga_rejects_bad_config():
    H = W = 16
    _, t, m = _problem(H, W, 0)
    init = ga.new_population(4, 3, H, W, MIN_S, MAX_S, np.random.default_rng(0))
    with pytest.raises(AssertionError):
        DeviceGA(t, m, init, tour_k=0, elite_k=1, cxpb=0.5, mutpb=0.1, min_scale_splats=MIN_S,
                 max_scale_splats=MAX_S, **CFG)
    with pytest.raises(AssertionError):
        DeviceGA(t, m, init, tour_k=2, elite_k=5, cxpb=0.5, mutpb=0.1, min_scale_splats=MIN_S,
                 max_scale_splats=MAX_S, **CFG)


# ---- device-resident SA neighbours (ggs_sa_*) -------------------------------------------------
def _sa(target, H, W, N, **kw):
    from ggs import annealing as A
    base = dict(mutpb=0.2, mut_sigma_max=CFG["mut_sigma_max"], mut_sigma_min=CFG["mut_sigma_min"],
                sigma_schedule="cosine", min_scale_splats=MIN_S, max_scale_splats=MAX_S,
                k_sigma=3.0, mask_strength=0.7, boost_only=False, iterations=6, temp0=2e-3,
                temp_schedule="cosine", tries_per_iter=4, progress=False, return_state=True)
    base.update(kw)
    return A.simulated_annealing(target, H, W, "cuda", n_splats=N, **base)


@pytest.mark.parametrize("H,W,N,tries,boost,spec", [(40, 40, 17, 4, False, None),
                                                     (64, 48, 300, 3, True, 1),
                                                     (32, 32, 1, 5, False, 5),
                                                     (48, 48, 2, 8, False, None),
                                                     # >= 1024 splats: 1024-thread variation
                                                     # workgroups, prep unfused, N > 512 raster
                                                     (64, 64, 1100, 3, False, None)])
def test_device_sa_matches_host_sa_with_same_draws(H, W, N, tries, boost, spec):
    target, _, _ = _problem(H, W, 5)
    init = ga.new_population(1, N, H, W, MIN_S, MAX_S, np.random.default_rng(N))[0]
    kw = dict(tries_per_iter=tries, boost_only=boost, speculate=spec, init_individual=init)
    hb, hf, hs = _sa(target, H, W, N, backend="host", seed=3, **kw)
    db, df, ds = _sa(target, H, W, N, backend="device", draws=ga.NumpyDraws(3), **kw)
    np.testing.assert_array_equal(db, hb)
    np.testing.assert_array_equal(ds["current"], hs["current"])
    assert df == hf and ds["curves"] == hs["curves"]
    assert all(ds["stats"][k] == hs["stats"][k] for k in ("evaluated", "tries", "launches"))


def test_device_sa_replays_reference_draws():
    from test_ga import ReplayDraws
    from test_sa import _case
    for name in ("cos", "exp", "log", "lin", "cau"):
        c = _case(name)
        iters, tries, T0, mutpb, boost = c["cfg"]
        b, f, st = _sa(c["target"], c["H"], c["W"], c["N"], mutpb=float(mutpb),
                       boost_only=bool(boost), iterations=int(iters), temp0=float(T0),
                       temp_schedule=str(c["sched"]), tries_per_iter=int(tries),
                       draws=ReplayDraws(c), init_individual=c["init"], backend="device")
        np.testing.assert_array_equal(b, c["best"], err_msg=name)
        assert f == pytest.approx(float(c["best_fit"]), rel=1e-5)
        for key in ("best", "current"):
            np.testing.assert_allclose(st["curves"][key], c[f"curve__{key}"], rtol=1e-5)


def test_device_sa_philox_width_invariant_and_improves():
    H = W = 96
    target, t, m = _problem(H, W, 6)
    init = ga.new_population(1, 64, H, W, MIN_S, MAX_S, np.random.default_rng(0))[0]
    outs = [_sa(target, H, W, 64, backend="device", seed=21, speculate=s, iterations=25,
                tries_per_iter=8, temp0=1e-4, init_individual=init) for s in (1, 3, None)]
    for b, f, st in outs[1:]:
        np.testing.assert_array_equal(b, outs[0][0])
        assert f == outs[0][1] and st["curves"] == outs[0][2]["curves"]
    b, f, st = outs[0]
    c = st["curves"]["best"]
    assert c[-1] < c[0] and all(y <= x for x, y in zip(c, c[1:]))
    assert float(ggs.fitness(b[None], t, H, W, 3.0, weight_mask=m)[0]) == f


@pytest.mark.parametrize("H,W,N,mutpb,boost", [(200, 150, 64, 0.002, False),
                                               (256, 256, 300, 0.05, True),
                                               (130, 260, 40, 0.02, False)])
def test_device_sa_incremental_equals_full_rerender(H, W, N, mutpb, boost):
    """Dirty-strip evaluation (only strips a changed splat touches) gives the
    full re-render's energies bit for bit, so the whole run is identical."""
    target, _, _ = _problem(H, W, 9)
    init = ga.new_population(1, N, H, W, MIN_S, MAX_S, np.random.default_rng(3))[0]
    kw = dict(mutpb=mutpb, boost_only=boost, iterations=12, tries_per_iter=6, temp0=1e-3,
              backend="device", seed=17, init_individual=init)
    b1, f1, s1 = _sa(target, H, W, N, incremental=True, **kw)
    b0, f0, s0 = _sa(target, H, W, N, incremental=False, **kw)
    np.testing.assert_array_equal(b1, b0)
    np.testing.assert_array_equal(s1["current"], s0["current"])
    assert f1 == f0 and s1["curves"] == s0["curves"]
    assert s1["stats"]["proposed"] == s1["stats"]["evaluated"] > 0
    assert 0 < s1["stats"]["changed_splats"] <= s1["stats"]["proposed"] * N


def test_device_sa_dirty_rules_equal_full_rerender(monkeypatch):
    """The two dirty-splat rules (GGS_SA_DIRTY_RULE, read at session creation):
    a splat is changed when its raster record differs (1, the default) or when any
    gene differs bitwise (0).  Both runs equal the full re-render bit for bit; the
    record rule never marks more splats (an unchanged record renders the same)."""
    H = W = 256
    N = 300
    target, _, _ = _problem(H, W, 21)
    init = ga.new_population(1, N, H, W, MIN_S, MAX_S, np.random.default_rng(21))[0]
    kw = dict(mutpb=0.01, iterations=10, tries_per_iter=6, temp0=1e-3, backend="device", seed=19,
              init_individual=init)
    b0, f0, s0 = _sa(target, H, W, N, incremental=False, **kw)
    changed = {}
    for rule in ("0", "1"):
        monkeypatch.setenv("GGS_SA_DIRTY_RULE", rule)
        b, f, st = _sa(target, H, W, N, incremental=True, **kw)
        np.testing.assert_array_equal(b, b0)
        np.testing.assert_array_equal(st["current"], s0["current"])
        assert f == f0 and st["curves"] == s0["curves"]
        changed[rule] = st["stats"]["changed_splats"]
    assert 0 < changed["1"] <= changed["0"], changed


@pytest.mark.parametrize("H,W,N,tries,spec,inc,iters", [(40, 40, 17, 4, None, False, 9),
                                                        (64, 48, 300, 3, 5, False, 7),
                                                        (48, 48, 2, 8, 1, False, 6),
                                                        (96, 80, 64, 6, None, True, 8),
                                                        # unfused prep (N > 1024), SAT raster
                                                        (64, 64, 1100, 3, 2, False, 4)])
def test_device_loop_matches_host_loop(H, W, N, tries, spec, inc, iters):
    """ggs_sa_run (iterations, Metropolis test and installs on the GPU) follows
    the host-driven loop over the same device proposer and the same Philox
    acceptance uniforms try for try: same states, energies and curves.  High T0
    so that acceptances (and re-proposed rounds) are frequent."""
    target, _, _ = _problem(H, W, 7)
    init = ga.new_population(1, N, H, W, MIN_S, MAX_S, np.random.default_rng(N + 1))[0]
    kw = dict(tries_per_iter=tries, speculate=spec, init_individual=init, iterations=iters,
              temp0=5e-2, backend="device", seed=11, incremental=inc)
    hb, hf, hs = _sa(target, H, W, N, loop="host", **kw)
    for chunk in (3, 256):
        db, df, ds = _sa(target, H, W, N, loop="device", chunk=chunk, **kw)
        np.testing.assert_array_equal(db, hb)
        np.testing.assert_array_equal(ds["current"], hs["current"])
        assert df == hf and ds["curves"] == hs["curves"]
        assert ds["current_fit"] == hs["current_fit"]
        assert ds["stats"]["tries"] == hs["stats"]["tries"] == iters * tries
        assert 0 < ds["stats"]["accepted"] and ds["stats"]["evaluated"] >= iters * tries


@pytest.mark.parametrize("tries,temp0", [(1, 5e-2), (4, 0.0)])
def test_device_loop_edge_schedules_match_host_loop(tries, temp0):
    """One try per iteration (every round is one neighbour of one iteration), and
    T0 = 0: the cosine schedule floors T at 1e-12 (annealing.py:37), so a rise dE
    of a float32 energy never passes the Metropolis test (annealing.py:133-145):
    the current energy never rises and equals the best curve."""
    H = W = 48
    N = 24
    target, _, _ = _problem(H, W, 13)
    init = ga.new_population(1, N, H, W, MIN_S, MAX_S, np.random.default_rng(13))[0]
    kw = dict(tries_per_iter=tries, init_individual=init, iterations=10, temp0=temp0, backend="device",
              seed=5)
    hb, hf, hs = _sa(target, H, W, N, loop="host", **kw)
    db, df, ds = _sa(target, H, W, N, loop="device", chunk=4, **kw)
    np.testing.assert_array_equal(db, hb)
    np.testing.assert_array_equal(ds["current"], hs["current"])
    assert df == hf and ds["curves"] == hs["curves"] and ds["current_fit"] == hs["current_fit"]
    assert ds["stats"]["tries"] == 10 * tries
    if temp0 == 0.0:
        cur = ds["curves"]["current"]
        assert all(y <= x for x, y in zip(cur, cur[1:])) and cur == ds["curves"]["best"]


def test_device_loop_width_invariant_low_temperature():
    """Rare acceptances: rounds span several iterations (width up to the cap);
    the trajectory does not depend on the width or the chunking."""
    H = W = 128
    target, t, m = _problem(H, W, 8)
    init = ga.new_population(1, 96, H, W, MIN_S, MAX_S, np.random.default_rng(2))[0]
    kw = dict(tries_per_iter=5, iterations=40, temp0=1e-6, backend="device", seed=5,
              init_individual=init)
    outs = [_sa(target, H, W, 96, speculate=s, chunk=c, **kw)
            for s, c in ((None, 256), (1, 7), (13, 256), (None, 1))]
    for b, f, st in outs[1:]:
        np.testing.assert_array_equal(b, outs[0][0])
        assert f == outs[0][1] and st["curves"] == outs[0][2]["curves"]
    # a round ends at an acceptance or after its width of tries, across iteration ends
    st13 = outs[2][2]["stats"]
    assert st13["launches"] <= st13["accepted"] + -(-200 // 13)
    assert outs[1][2]["stats"]["evaluated"] == outs[1][2]["stats"]["launches"]   # width 1
    b, f, _ = outs[0]
    assert float(ggs.fitness(b[None], t, H, W, 3.0, weight_mask=m)[0]) == f


def test_device_loop_rejects_mixed_driving():
    from ggs.ga_device import DeviceSA
    H = W = 32
    _, t, m = _problem(H, W, 1)
    init = ga.new_population(1, 8, H, W, MIN_S, MAX_S, np.random.default_rng(0))[0]
    sa = DeviceSA(t, m, init, max_tries=4, mutpb=0.1, schedule="cosine", min_scale_splats=MIN_S,
                  max_scale_splats=MAX_S, mut_sigma_max=CFG["mut_sigma_max"],
                  mut_sigma_min=CFG["mut_sigma_min"], seed=1)
    try:
        with pytest.raises(AssertionError):           # GGS_EINVAL
            sa.run(0, [1e-3], 1, 2, width=5)          # width above the capacity
        sa.run(0, [1e-3, 1e-3], 2, 2)
        with pytest.raises(AssertionError):
            sa.propose(0, 2, 0, 2)
    finally:
        sa.close()


def test_device_loop_incremental_equals_full_at_configs4_size():
    """configs[4] size (2048^2, 4,096 splats, 8 tries): the dirty-strip path (only
    strips a changed splat touches are rasterised, the rest keep the state's
    partials) gives the full re-render's run bit for bit, at a MUTPB low enough
    that most strips stay clean."""
    H = W = 2048
    target, _, _ = _problem(H, W, 4)
    init = ga.new_population(1, 4096, H, W, MIN_S, MAX_S, np.random.default_rng(7))[0]
    kw = dict(mutpb=2e-4, iterations=6, tries_per_iter=8, temp0=1e-3, backend="device", seed=3,
              init_individual=init)
    b1, f1, s1 = _sa(target, H, W, 4096, incremental=True, **kw)
    b0, f0, s0 = _sa(target, H, W, 4096, incremental=False, **kw)
    np.testing.assert_array_equal(b1, b0)
    np.testing.assert_array_equal(s1["current"], s0["current"])
    assert f1 == f0 and s1["curves"] == s0["curves"]
    assert 0 < s1["stats"]["changed_splats"] < s1["stats"]["proposed"] * 4096 // 4


@pytest.mark.parametrize("H,W,N", [(96, 80, 64), (128, 128, 200)])
def test_device_loop_incremental_switched_on_mid_run_equals_full(H, W, N):
    """a device loop run with incremental evaluation OFF accepts
    neighbours without installing their records / strip partials, so switching it
    ON afterwards must re-derive them (ggs_sa_set_incremental) before the dirty-
    strip test relies on them.  Session A: 6 iterations full, then incremental on,
    6 more; session B: full throughout, same seed and temperatures — identical
    curves, current and best states, bit for bit.  Also on -> off -> on, and on
    right after create (nothing to re-derive)."""
    from ggs.ga_device import DeviceSA
    target, t, m = _problem(H, W, 12)
    init = ga.new_population(1, N, H, W, MIN_S, MAX_S, np.random.default_rng(N))[0]
    temps = np.full(12, 5e-2)

    def session(inc0):
        return DeviceSA(t, m, init, max_tries=8, mutpb=0.05, min_scale_splats=MIN_S, max_scale_splats=MAX_S,
                        seed=23, incremental=inc0, **CFG)

    def drive(sa, plan):
        curves = []
        for (i0, i1), inc in plan:
            if inc is not None:
                ggs._lib.check(ggs._lib.lib.ggs_sa_set_incremental(sa.h, int(inc)), "set_incremental")
            curves.append(sa.run(i0, temps[i0:i1], 12, 4))
        cur, best, _ = sa.read()
        sa.close()
        return np.concatenate(curves), cur, best

    full = drive(session(False), [((0, 12), None)])
    for inc0, plan in ((False, [((0, 6), None), ((6, 12), True)]),
                       (True, [((0, 4), None), ((4, 8), False), ((8, 12), True)]),
                       (True, [((0, 12), None)])):
        got = drive(session(inc0), plan)
        for a, b in zip(got, full):
            np.testing.assert_array_equal(a, b)
