"""Golden fixtures for the GA layer (§8f next #1), made by running the REFERENCE.

Build container only (refuses to run without /root/reference).  The reference's
variation operators draw from torch's and Python's global RNGs, which a numpy
host cannot reproduce; so every draw the reference makes is RECORDED here (by
wrapping the `torch` / `random` module attributes of the reference modules —
no reference code is copied) and stored next to the reference's inputs and
outputs.  tests/test_ga.py replays the recorded draws through ggs/ga.py's
batched operators and requires identical results.

  ga_mutate.npz  mutate_individual (genetic.py:32-91): inputs, draws, outputs
  ga_loop.npz    genetic_approx (algorithm.py:17-195), 3 generations on CPU
                 (Triton interpreter renders): initial population, the Python
                 and torch draw streams, every fitness call's population and
                 values, final best and curves
  sa_loop.npz    simulated_annealing (annealing.py:47-190), same recording, for
                 three temperature schedules
"""
from __future__ import annotations

import os
import random as pyrandom
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
if not os.path.isdir(os.path.join(REF, "modules")):
    raise SystemExit("make_golden_ga.py: /root/reference is not present")

os.environ["TRITON_INTERPRET"] = "1"
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import modules.algorithm as A  # noqa: E402  (reference)
import modules.annealing as SA  # noqa: E402  (reference)
import modules.config as CFG  # noqa: E402  (reference)
import modules.fitness as F  # noqa: E402  (reference)
import modules.genetic as GEN  # noqa: E402  (reference)
from make_golden import ref_render_cpu  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
from ggs_oracle import synthetic_population  # noqa: E402  (input spec only)


class TorchTap:
    """Stands in for `torch` inside modules.genetic: forwards everything, logs
    the tensors returned by rand / randn_like / randint in call order."""

    def __init__(self):
        self.log = []

    def __getattr__(self, name):
        return getattr(torch, name)

    def rand(self, *a, **k):
        t = torch.rand(*a, **k)
        self.log.append(("rand", t.clone()))
        return t

    def randn_like(self, x, **k):
        t = torch.randn_like(x, **k)
        self.log.append(("randn", t.clone()))
        return t

    def randint(self, *a, **k):
        t = torch.randint(*a, **k)
        self.log.append(("randint", t.clone()))
        return t


class RandomTap:
    """Stands in for `random` inside modules.genetic / modules.algorithm."""

    def __init__(self, seed):
        self.r = pyrandom.Random(seed)
        self.log = []

    def random(self):
        v = self.r.random()
        self.log.append(("random", v))
        return v

    def randrange(self, n):
        v = self.r.randrange(n)
        self.log.append(("randrange", v))
        return v

    def shuffle(self, x):
        perm = list(range(len(x)))
        self.r.shuffle(perm)
        orig = list(x)
        x[:] = [orig[i] for i in perm]
        self.log.append(("shuffle", perm))


def split_mutation_draws(log, N, mutpb):
    """Assign one mutate_individual's torch draws to named slots (genetic.py:37-91)."""
    it = iter(log)
    d = {}
    for key in ("u_xy", "u_ab", "u_t", "u_rgb", "u_a"):
        kind, t = next(it)
        assert kind == "rand"
        d[key] = t.numpy()
    p = np.float32(mutpb)
    need = {"k_color": not ((d["u_rgb"] < p).any() or (d["u_a"] < p).any()),
            "k_xy": not (d["u_xy"] < p).any(), "k_ab": not (d["u_ab"] < p).any(),
            "k_t": not (d["u_t"] < p).any()}
    for key in ("k_color", "k_xy", "k_ab", "k_t"):          # _ensure_one_true order
        if need[key]:
            kind, t = next(it)
            assert kind == "randint"
            d[key] = int(t.item())
        else:
            d[key] = -1
    for key in ("n_xy", "n_ab", "n_t", "n_rgba"):
        kind, t = next(it)
        assert kind == "randn"
        d[key] = t.numpy()
    rest = list(it)
    d["swap_i"] = int(rest[0][1].item()) if N >= 2 else -1
    d["swap_pick"] = int(rest[1][1].item()) if len(rest) > 1 else -1
    assert len(rest) <= 2
    return d


def mutate_fixture():
    out = {}
    cases = [("p05", 16, 0.05, 3, 10), ("p30", 24, 0.30, 7, 10), ("p01", 6, 0.01, 0, 5),
             ("n2", 2, 0.2, 4, 4), ("big", 64, 0.05, 50, 500)]
    H, W = 48, 40
    for name, N, mutpb, gen, total in cases:
        pop = synthetic_population(6, N, H, W, seed=N * 7 + gen)
        ins, outs, draws = [], [], []
        for ind in pop:
            tap = TorchTap()
            GEN.torch = tap
            x = torch.from_numpy(ind.copy())
            y = GEN.mutate_individual(x, is_elite=False, gen=gen, total_gens=total,
                                      schedule=CFG.SCHEDULE, mut_sigma_max=CFG.MUT_SIGMA_MAX,
                                      mut_sigma_min=CFG.MUT_SIGMA_MIN, mutpb=mutpb, H=H, W=W,
                                      min_scale_splats=CFG.MIN_SCALE_SPLATS,
                                      max_scale_splats=CFG.MAX_SCALE_SPLATS)
            GEN.torch = torch
            ins.append(ind)
            outs.append(y.numpy().copy())
            draws.append(split_mutation_draws(tap.log, N, mutpb))
        out[f"{name}__in"] = np.stack(ins)
        out[f"{name}__out"] = np.stack(outs)
        out[f"{name}__cfg"] = np.array([N, mutpb, gen, total, H, W], np.float64)
        for key in draws[0]:
            out[f"{name}__{key}"] = np.stack([np.asarray(d[key]) for d in draws])
    np.savez_compressed(os.path.join(HERE, "ga_mutate.npz"), **out)


def _streams(out, rtap, ttap, pre=""):
    """Python stream: kinds 0 random, 1 randrange, 2 shuffle (perm stored
    separately); torch stream: kinds 0 rand, 1 randn, 2 randint, flattened."""
    py_kind, py_val, perms = [], [], []
    for kind, v in rtap.log:
        if kind == "shuffle":
            py_kind.append(2)
            py_val.append(len(perms))
            perms.append(v)
        else:
            py_kind.append(0 if kind == "random" else 1)
            py_val.append(v)
    out[pre + "py_kind"] = np.array(py_kind, np.int64)
    out[pre + "py_val"] = np.array(py_val, np.float64)
    out[pre + "py_perms"] = np.array(perms, np.int64) if perms else np.zeros((0, 0), np.int64)
    t_kind, t_shape, t_off, flat = [], [], [], []
    off = 0
    for kind, t in ttap.log:
        t_kind.append({"rand": 0, "randn": 1, "randint": 2}[kind])
        a = t.numpy().astype(np.float64).ravel()
        t_shape.append(list(t.shape) + [0] * (2 - t.dim()) if t.dim() <= 2 else list(t.shape))
        t_off.append(off)
        flat.append(a)
        off += a.size
    out[pre + "t_kind"] = np.array(t_kind, np.int64)
    out[pre + "t_shape"] = np.array(t_shape, np.int64)
    out[pre + "t_off"] = np.array(t_off + [off], np.int64)
    out[pre + "t_flat"] = np.concatenate(flat) if flat else np.zeros(0)


def sa_fixture():
    """simulated_annealing on CPU with recorded draws; cases differ in schedule,
    T0 (random acceptance exercised) and tries per iteration."""
    H, W, N = 32, 28, 10
    target = np.random.default_rng(9).uniform(0, 255, (36, 30, 3)).astype(np.float32)
    cases = [("cos", "cosine", 2e-3, 3, 6, 0.2), ("exp", "exp", 5e-2, 2, 5, 0.3),
             ("log", "log", 0.0, 4, 3, 0.1), ("lin", "linear", 1e-2, 1, 6, 0.5),
             ("cau", "cauchy", 1e-2, 2, 3, 0.2)]
    out = {"target": target, "dims": np.array([H, W, N], np.int64)}
    for name, sched, T0, tries, iters, mutpb in cases:
        torch.manual_seed(7)
        rtap = RandomTap(11)
        ttap = TorchTap()
        SA.random = rtap
        GEN.random = rtap
        GEN.torch = ttap
        F.render_splats_rgb_triton = ref_render_cpu
        rec = {"init": None, "calls": [], "curves": None}

        def new_individual(*a, **k):
            ind = torch.from_numpy(synthetic_population(1, N, H, W, seed=13)[0])
            rec["init"] = ind.numpy().copy()
            return ind

        def fitness_population(population, *a, **k):
            vals = F.fitness_population(population, *a, **k)
            rec["calls"].append((np.stack([p.numpy() for p in population]), np.asarray(vals)))
            return vals

        def save_curves_csv(curves, path):
            rec["curves"] = {k: np.asarray(v, np.float64) for k, v in curves.items()}

        SA.new_individual = new_individual
        SA.fitness_population = fitness_population
        SA.prewarm_renderer = lambda *a, **k: None
        SA.save_curves_csv = save_curves_csv
        SA.save_loss_curve_png = lambda *a, **k: None
        best, best_fit = SA.simulated_annealing(
            torch.from_numpy(target), H=H, W=W, device="cpu", n_splats=N, mutpb=mutpb,
            mut_sigma_max=CFG.MUT_SIGMA_MAX, mut_sigma_min=CFG.MUT_SIGMA_MIN,
            sigma_schedule=CFG.SCHEDULE, min_scale_splats=CFG.MIN_SCALE_SPLATS,
            max_scale_splats=CFG.MAX_SCALE_SPLATS, k_sigma=3.0, mask_strength=0.7,
            boost_only=name == "exp", iterations=iters, temp0=T0, temp_schedule=sched,
            tries_per_iter=tries, loss_csv_path="unused.csv")
        pre = name + "__"
        out[pre + "cfg"] = np.array([iters, tries, T0, mutpb, name == "exp"], np.float64)
        out[pre + "sched"] = np.array(sched)
        out[pre + "init"] = rec["init"]
        out[pre + "best"] = best.numpy()
        out[pre + "best_fit"] = np.float64(best_fit)
        out[pre + "n_calls"] = np.int64(len(rec["calls"]))
        for i, (pop, vals) in enumerate(rec["calls"]):
            out[pre + f"call{i}__pop"] = pop
            out[pre + f"call{i}__fit"] = vals
        for k, v in rec["curves"].items():
            out[pre + f"curve__{k}"] = v
        _streams(out, rtap, ttap, pre)
        print("sa", name, "best_fit", best_fit, "calls", len(rec["calls"]),
              "accept draws", sum(1 for k, _ in rtap.log if k == "random"))
    GEN.torch = torch
    np.savez_compressed(os.path.join(HERE, "sa_loop.npz"), **out)


def loop_fixture():
    H = W = 32
    P, N, G = 8, 8, 3
    torch.manual_seed(42)
    target = np.random.default_rng(3).uniform(0, 255, (40, 36, 3)).astype(np.float32)
    rtap = RandomTap(42)
    ttap = TorchTap()
    A.random = rtap
    GEN.random = rtap
    GEN.torch = ttap
    F.render_splats_rgb_triton = ref_render_cpu
    rec = {"init": None, "calls": [], "curves": None}

    def new_population(*a, **k):
        pop = F.torch.from_numpy(synthetic_population(P, N, H, W, seed=77))
        rec["init"] = pop.numpy().copy()
        return pop

    def fitness_population(population, *a, **k):
        vals = F.fitness_population(population, *a, **k)
        rec["calls"].append((np.stack([p.numpy() for p in population]), np.asarray(vals)))
        return vals

    def save_curves_csv(curves, path):
        rec["curves"] = {k: np.asarray(v, np.float64) for k, v in curves.items()}

    A.new_population = new_population
    A.fitness_population = fitness_population
    A.prewarm_renderer = lambda *a, **k: None
    A.save_curves_csv = save_curves_csv
    A.save_loss_curve_png = lambda *a, **k: None
    best, best_fit = A.genetic_approx(
        torch.from_numpy(target), H=H, W=W, device="cpu", pop_size=P, n_splats=N,
        generations=G, tour_k=2, elite_k=2, cxpb=0.5, mutpb=0.2,
        mut_sigma_max=CFG.MUT_SIGMA_MAX, mut_sigma_min=CFG.MUT_SIGMA_MIN,
        schedule=CFG.SCHEDULE, min_scale_splats=CFG.MIN_SCALE_SPLATS,
        max_scale_splats=CFG.MAX_SCALE_SPLATS, k_sigma=3.0, mask_strength=0.7,
        boost_only=False, loss_csv_path="unused.csv")
    out = {"target": target, "cfg": np.array([H, W, P, N, G, 2, 2, 0.5, 0.2], np.float64),
           "init": rec["init"], "best": best.numpy(), "best_fit": np.float64(best_fit)}
    for i, (pop, vals) in enumerate(rec["calls"]):
        out[f"call{i}__pop"] = pop
        out[f"call{i}__fit"] = vals
    out["n_calls"] = np.int64(len(rec["calls"]))
    for k, v in rec["curves"].items():
        out[f"curve__{k}"] = v
    # python stream: kinds 0 random, 1 randrange, 2 shuffle (perm stored separately)
    py_kind, py_val, perms = [], [], []
    for kind, v in rtap.log:
        if kind == "shuffle":
            py_kind.append(2)
            py_val.append(len(perms))
            perms.append(v)
        else:
            py_kind.append(0 if kind == "random" else 1)
            py_val.append(v)
    out["py_kind"] = np.array(py_kind, np.int64)
    out["py_val"] = np.array(py_val, np.float64)
    out["py_perms"] = np.array(perms, np.int64)
    # torch stream: kinds 0 rand, 1 randn, 2 randint; flattened values with offsets
    t_kind, t_shape, t_off, flat = [], [], [], []
    off = 0
    for kind, t in ttap.log:
        t_kind.append({"rand": 0, "randn": 1, "randint": 2}[kind])
        a = t.numpy().astype(np.float64).ravel()
        t_shape.append(list(t.shape) + [0] * (2 - t.dim()) if t.dim() <= 2 else list(t.shape))
        t_off.append(off)
        flat.append(a)
        off += a.size
    out["t_kind"] = np.array(t_kind, np.int64)
    out["t_shape"] = np.array(t_shape, np.int64)
    out["t_off"] = np.array(t_off + [off], np.int64)
    out["t_flat"] = np.concatenate(flat) if flat else np.zeros(0)
    np.savez_compressed(os.path.join(HERE, "ga_loop.npz"), **out)
    print("ga loop: best_fit", best_fit, "calls", len(rec["calls"]))


if __name__ == "__main__":
    which = sys.argv[1:] or ["mutate", "loop", "sa"]
    if "mutate" in which:
        mutate_fixture()
    if "loop" in which:
        loop_fixture()
    if "sa" in which:
        sa_fixture()
    print("done")
