"""The batched GA layer (ggs/ga.py) against the REFERENCE's GA, draw for draw.

tests/golden/make_golden_ga.py ran the reference's mutate_individual and a
3-generation genetic_approx on CPU while recording every random draw it made
(torch and Python RNG).  Here those draws are replayed through ggs/ga.py's
batched operators: the mutated genomes, every generation's offspring, the
elites, the best individual and the curves must come out identical.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import load_golden
from ggs import ga

CFG = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0,
                          "alpha": 25.0},
           mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0,
                          "alpha": 2.0},
           schedule="cosine")          # reference modules/config.py:22-43
MIN_S, MAX_S = 3.0, 0.1                # config.py:16-17
DRAW_KEYS = ("u_xy", "u_ab", "u_t", "u_rgb", "u_a", "k_color", "k_xy", "k_ab", "k_t",
             "n_xy", "n_ab", "n_t", "n_rgba", "swap_i", "swap_pick")


def _mutate_cases():
    d = load_golden("ga_mutate.npz")
    return sorted({k.split("__")[0] for k in d.files})


@pytest.mark.parametrize("case", _mutate_cases())
def test_mutate_matches_reference(case):
    d = load_golden("ga_mutate.npz")
    N, mutpb, gen, total, H, W = d[f"{case}__cfg"]
    draws = {k: d[f"{case}__{k}"] for k in DRAW_KEYS}
    draws["swap_u"] = np.zeros(len(draws["swap_i"]))
    G = d[f"{case}__in"].copy()
    out = ga.mutate_batch(G, draws, int(gen), int(total), CFG["schedule"], CFG["mut_sigma_max"],
                          CFG["mut_sigma_min"], float(mutpb), int(H), int(W), MIN_S, MAX_S)
    np.testing.assert_array_equal(out, d[f"{case}__out"])


class ReplayDraws:
    """Serves the reference's recorded draw streams to ggs.ga in its batch shapes."""

    def __init__(self, d):
        self.d = d
        self.pi = 0                     # python stream cursor
        self.ti = 0                     # torch stream cursor

    # python stream ---------------------------------------------------------------
    def _py(self, kind):
        k = int(self.d["py_kind"][self.pi])
        v = self.d["py_val"][self.pi]
        assert k == kind, (k, kind, self.pi)
        self.pi += 1
        return v

    def tournament(self, P, k):
        return np.array([[int(self._py(1)) for _ in range(k)] for _ in range(P)])

    def shuffle(self, P):
        return self.d["py_perms"][int(self._py(2))]

    def uniform(self, n):
        return np.array([self._py(0) for _ in range(n)])

    # torch stream ----------------------------------------------------------------
    def _t(self, kind=None):
        k = int(self.d["t_kind"][self.ti])
        if kind is not None:
            assert k == kind, (k, kind, self.ti)
        a, b = self.d["t_off"][self.ti], self.d["t_off"][self.ti + 1]
        shape = [s for s in self.d["t_shape"][self.ti] if s > 0]
        self.ti += 1
        return k, self.d["t_flat"][a:b].reshape(shape)

    def _peek(self):
        return int(self.d["t_kind"][self.ti]) if self.ti < len(self.d["t_kind"]) else -1

    def _mutation_one(self, N, mutpb):
        r = {}
        for key in ("u_xy", "u_ab", "u_t", "u_rgb", "u_a"):
            r[key] = self._t(0)[1].astype(np.float32)
        p = np.float32(mutpb)
        need = {"k_color": not ((r["u_rgb"] < p).any() or (r["u_a"] < p).any()),
                "k_xy": not (r["u_xy"] < p).any(), "k_ab": not (r["u_ab"] < p).any(),
                "k_t": not (r["u_t"] < p).any()}
        for key in ("k_color", "k_xy", "k_ab", "k_t"):
            r[key] = int(self._t(2)[1].ravel()[0]) if need[key] else 0
        for key in ("n_xy", "n_ab", "n_t", "n_rgba"):
            r[key] = self._t(1)[1].astype(np.float32)
        r["swap_i"] = int(self._t(2)[1].ravel()[0])
        r["swap_pick"] = int(self._t(2)[1].ravel()[0]) if self._peek() == 2 else -1
        r["swap_u"] = 0.0
        return r

    def mutation(self, n, N, mutpb):          # SA: the tries of one iteration
        muts = [self._mutation_one(N, mutpb) for _ in range(n)]
        return {k: np.stack([np.asarray(m[k]) for m in muts]) for k in muts[0]}

    def accept(self):                         # annealing.py:142 random.random()
        return float(self._py(0))

    def generation(self, cx, n_off, N, mutpb):
        masks, muts = [], []
        for i, c in enumerate(cx):
            if c:
                masks.append(self._t(0)[1].astype(np.float32))
            muts.append(self._mutation_one(N, mutpb))
            if 2 * i + 1 < n_off:
                muts.append(self._mutation_one(N, mutpb))
        mut = {k: np.stack([np.asarray(m[k]) for m in muts]) for k in muts[0]}
        cxu = np.stack(masks) if masks else np.zeros((0, N, 1), np.float32)
        return cxu, mut


def test_ga_loop_matches_reference():
    d = load_golden("ga_loop.npz")
    H, W, P, N, G, tour_k, elite_k, cxpb, mutpb = d["cfg"]
    H, W, P, N, G, tour_k, elite_k = (int(v) for v in (H, W, P, N, G, tour_k, elite_k))
    calls = []

    def evaluate(pop):                        # the reference's own fitness values
        k = len(calls)
        ref_call = 0 if k == 0 else 2 * k - 1  # skip the reference's elite re-evaluations
        # offspring: only the P - elite_k that survive are evaluated (the first ones)
        n = len(pop)
        assert n == (P if k == 0 else P - max(1, elite_k))
        np.testing.assert_array_equal(pop, d[f"call{ref_call}__pop"][:n], err_msg=f"call {ref_call}")
        calls.append(ref_call)
        return d[f"call{ref_call}__fit"][:n].astype(np.float32)

    best, best_fit, st = ga.genetic_approx(
        d["target"], H, W, "cuda", pop_size=P, n_splats=N, generations=G, tour_k=tour_k,
        elite_k=elite_k, cxpb=float(cxpb), mutpb=float(mutpb), min_scale_splats=MIN_S,
        max_scale_splats=MAX_S, k_sigma=3.0, mask_strength=0.7, boost_only=False,
        draws=ReplayDraws(d), evaluate=evaluate, init_population=d["init"], progress=False,
        return_state=True, **CFG)
    assert len(calls) == G + 1
    # the elites the reference re-evaluated are exactly our carried-over survivors
    last_elites = d[f"call{2 * G}__pop"]
    np.testing.assert_array_equal(st["population"][:elite_k], last_elites)
    np.testing.assert_array_equal(st["fitness"][:elite_k], d[f"call{2 * G}__fit"].astype(np.float32))
    np.testing.assert_array_equal(best, d["best"])
    assert best_fit == float(d["best_fit"])
    for key in ("best", "mean", "median"):
        np.testing.assert_allclose(st["curves"][key], d[f"curve__{key}"], rtol=1e-12, atol=0)


def test_numpy_draws_ga_runs_and_improves():
    """Self-consistency with the default draw source and a CPU oracle evaluator."""
    import ggs_oracle as O
    H = W = 24
    rng = np.random.default_rng(0)
    target = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    from ggs.mask import compute_importance_mask
    mask = compute_importance_mask(target, H, W, smooth=3, strength=0.7)

    def evaluate(pop):
        return O.fitness_many(list(pop), target, H, W, 3.0, weight_mask=mask).astype(np.float32)

    best, best_fit, st = ga.genetic_approx(
        target, H, W, "cuda", pop_size=10, n_splats=6, generations=6, tour_k=2, elite_k=2,
        cxpb=0.3, mutpb=0.2, min_scale_splats=MIN_S, max_scale_splats=MAX_S, k_sigma=3.0,
        mask_strength=0.7, boost_only=False, seed=5, evaluate=evaluate, progress=False,
        return_state=True, **CFG)
    c = st["curves"]["best"]
    assert len(c) == 7 and all(b <= a for a, b in zip(c, c[1:]))
    assert best.shape == (6, 9) and best_fit == c[-1]
    np.testing.assert_allclose(evaluate(best[None])[0], best_fit, rtol=1e-6)
    # operators keep the genome in range (utils.py:35-45)
    P = st["population"]
    assert (P[..., 0:2] >= 0).all() and (P[..., 0:2] <= 1).all()
    assert (P[..., 4] >= -np.pi - 1e-6).all() and (P[..., 4] < np.pi + 1e-6).all()
    assert (P[..., 5:9] >= 0).all() and (P[..., 5:9] <= 255).all()


def test_tournament_first_min_and_wrap():
    fits = np.array([3.0, 1.0, 1.0, 2.0])
    idx = np.array([[0, 3], [2, 1], [1, 2], [3, 3]])
    np.testing.assert_array_equal(ga.tournament(fits, idx), [3, 2, 1, 3])
    th = np.array([-4.0, 3.2, np.pi, -np.pi, 0.0], np.float32)
    w = ga.wrap_angle(th)
    assert w.dtype == np.float32 and (w >= -np.pi - 1e-6).all() and (w < np.pi + 1e-6).all()
