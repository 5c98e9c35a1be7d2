"""Simulated annealing (ggs/annealing.py) against the REFERENCE's
simulated_annealing (annealing.py:47-190), draw for draw.

tests/golden/make_golden_ga.py ran the reference on CPU for five temperature
schedules while recording its torch and Python draws, every fitness call and
the curves.  Replaying those draws:
* width 1 (sequential, the reference's schedule): every evaluated neighbour is
  the reference's genome bit for bit, in the same order;
* batched speculation (width = tries, and adaptive): the same accepted states,
  best individual and curves — speculative neighbours the reference never
  evaluated are discarded before they can influence anything.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import load_golden
from ggs import annealing as A
from test_ga import CFG, MAX_S, MIN_S, ReplayDraws

CASES = ["cos", "exp", "log", "lin", "cau"]


def _case(name):
    d = load_golden("sa_loop.npz")
    pre = name + "__"
    c = {k[len(pre):]: d[k] for k in d.files if k.startswith(pre)}
    c["target"], (c["H"], c["W"], c["N"]) = d["target"], (int(v) for v in d["dims"])
    return c


def _run(c, speculate, evaluate):
    iters, tries, T0, mutpb, boost = c["cfg"]
    return A.simulated_annealing(
        c["target"], c["H"], c["W"], "cuda", n_splats=c["N"], mutpb=float(mutpb),
        mut_sigma_max=CFG["mut_sigma_max"], mut_sigma_min=CFG["mut_sigma_min"],
        sigma_schedule=CFG["schedule"], min_scale_splats=MIN_S, max_scale_splats=MAX_S,
        k_sigma=3.0, mask_strength=0.7, boost_only=bool(boost), iterations=int(iters),
        temp0=float(T0), temp_schedule=str(c["sched"]), tries_per_iter=int(tries),
        draws=ReplayDraws(c), evaluate=evaluate, init_individual=c["init"], progress=False,
        return_state=True, speculate=speculate)


def _check_result(c, out):
    best, best_fit, st = out
    np.testing.assert_array_equal(best, c["best"])
    assert best_fit == float(c["best_fit"])
    for key in ("best", "current"):
        np.testing.assert_array_equal(np.asarray(st["curves"][key]), c[f"curve__{key}"])


@pytest.mark.parametrize("name", CASES)
def test_sa_sequential_matches_reference(name):
    c = _case(name)
    calls = []

    def evaluate(G):
        i = len(calls)
        assert len(G) == 1
        np.testing.assert_array_equal(G[0], c[f"call{i}__pop"][0], err_msg=f"call {i}")
        calls.append(i)
        return c[f"call{i}__fit"].astype(np.float32)

    out = _run(c, 1, evaluate)
    assert len(calls) == int(c["n_calls"])
    _check_result(c, out)


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("speculate", [None, 8])
def test_sa_batched_speculation_matches_reference(name, speculate):
    c = _case(name)
    known = {c[f"call{i}__pop"][0].tobytes(): float(c[f"call{i}__fit"][0])
             for i in range(int(c["n_calls"]))}

    def evaluate(G):          # neighbours the reference never evaluated get NaN
        return np.array([known.get(g.tobytes(), np.nan) for g in G], np.float32)

    out = _run(c, speculate, evaluate)
    _check_result(c, out)
    st = out[2]["stats"]
    assert st["evaluated"] >= int(c["n_calls"]) - 1


def test_temp_schedules():
    for kind in ("exp", "linear", "cosine", "log", "cauchy", "other"):
        vals = [A.temp_schedule(kind, 1e-3, i, 10) for i in range(11)]
        assert all(v > 0 for v in vals) and vals[0] == pytest.approx(1e-3)
        assert all(b <= a for a, b in zip(vals, vals[1:]))
    assert A.temp_schedule("exp", 1.0, 10, 10) == pytest.approx(0.01)


def test_device_loop_width_sizes_rounds_to_the_grid():
    """A device-loop round holds enough neighbours for ~10 rounds of raster wave
    slots (2048^2: 16 of 2,048 strips; 512^2: 64 of 256), never fewer than one
    iteration's tries."""
    assert A.device_loop_width(2048, 2048, 8) == 16
    assert A.device_loop_width(512, 512, 8) == 64
    assert A.device_loop_width(4096, 4096, 8) == 8          # 8,192 strips: one iteration's tries
    assert A.device_loop_width(4096, 4096, 20) == 20
    assert A.device_loop_width(16, 16, 1) == 64


@pytest.mark.parametrize("kw", [dict(loop="device", backend="host"),
                                dict(loop="bogus", backend="host"),
                                dict(loop="device", backend="device", draws=object()),
                                dict(backend="bogus")])
def test_sa_rejects_inconsistent_loop_arguments(kw):
    """loop='device' needs the device backend and in-kernel draws; unknown loop /
    backend names raise before any evaluation."""
    H = W = 16
    target = np.random.default_rng(0).uniform(0, 255, (H, W, 3)).astype(np.float32)

    def never(G):                                  # the checks come first
        raise AssertionError("evaluated")
    with pytest.raises(ValueError):
        A.simulated_annealing(target, H, W, "cuda", 4, 0.1, CFG["mut_sigma_max"],
                              CFG["mut_sigma_min"], "cosine", MIN_S, MAX_S, 3.0, 0.7, False, 2,
                              1e-3, "cosine", 2, evaluate=never if kw.get("backend") == "host" else None,
                              progress=False, **kw)


def test_device_loop_batching_rule_is_bounded():
    """ggs_sa_run's rounds per host sync (ggs_sa_rounds_per_sync, pure host
    arithmetic): enough rounds to finish the chunk at the expected consumption
    (never past it), at least one, and never more than GGS_SA_MAX_ROUNDS_PER_SYNC
    — an unbounded batch (~1,000 rounds = 4,000 queued dispatches at high
    acceptance) crashed the launch under rocprofv3 --pmc (docs/EXPERIMENTS.md §9)."""
    import re
    from conftest import REPO
    from ggs import lib
    cap = int(re.search(r"#define GGS_SA_MAX_ROUNDS_PER_SYNC (\d+)",
                        open(f"{REPO}/include/ggs.h").read()).group(1))
    assert 16 <= cap <= 256
    f = lib.ggs_sa_rounds_per_sync
    for remaining in (0, 1, 7, 8, 63, 64, 65, 2048, 16_000, 2**31 - 1):
        for est in (-3, 0, 1, 2, 3, 16, 64, 10_000):
            R = f(remaining, est)
            e = max(1, est)
            assert 1 <= R <= cap
            assert R == max(1, min(cap, -(-max(remaining, 0) // e)))
            assert (R - 1) * e < max(remaining, 1)      # the batch never starts a round past the chunk
    assert f(2048, 2) == cap and f(16_000, 16) == cap   # the crashing regimes are capped
