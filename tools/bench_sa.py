"""SA throughput at BASELINE configs[4] (run_sags.py: 2048x2048, 4096 splats,
SA_TRIES_PER_ITER=8, MUTPB=0.05, T0=1e-3 cosine): iterations/s of
ggs.annealing.simulated_annealing over the SA loop alone (stats["loop_s"]: the
iteration loop's own wall time; setup — target prep, importance mask, initial
evaluation, ~0.9 s at 2048^2 — is reported separately.  Round 1 subtracted a
separately timed setup run instead, and its ±50 ms jitter swamped the ~0.2 s loop):
* host / sequential: numpy mutation, one host-API launch per try (the
  reference's schedule);
* host / speculative: numpy mutation, batched tries;
* device / host loop: state resident in HBM, in-kernel mutation (Philox),
  batched tries, one 4-byte-per-try readback and host acceptance test per batch;
* device / device loop (ggs_sa_run, the default): acceptance walk and state
  installs on the GPU too, rounds spanning iterations, one host sync per batch
  of rounds; "full" re-rasterises every strip, "incremental" only the strips a
  changed splat touches.  Timed --repeat times over --dev-iters iterations.

usage: python tools/bench_sa.py [--iters 20] [--dev-iters 200] [--repeat 3] [--size 2048]
                                [--splats 4096] [--tries 8] [--only device_loop_full]"""
import argparse, json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "genetic-gaussian-splats_amd"))
from ggs import annealing as A
from ggs import ga

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--size", type=int, default=2048)
ap.add_argument("--splats", type=int, default=4096)
ap.add_argument("--tries", type=int, default=8)
ap.add_argument("--mutpb", type=float, default=0.05)
ap.add_argument("--dev-iters", type=int, default=200)
ap.add_argument("--repeat", type=int, default=3)
ap.add_argument("--temp0", type=float, default=1e-3)
ap.add_argument("--speculate", type=int, default=0,
                help="fixed round width for the device variants (0: adaptive, the default)")
ap.add_argument("--only", default="")
ap.add_argument("--warm", type=int, default=0,
                help="start from the best state of a --warm-iteration device run (T0 1e-3), so the "
                     "timed runs see the late-run regime where acceptances are rare")
a = ap.parse_args()
H = W = a.size
target = np.random.default_rng(0).uniform(0, 1, (H, W, 3)).astype(np.float32)
init = ga.new_population(1, a.splats, H, W, 3.0, 0.1, np.random.default_rng(1))[0]
cfg = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0, "alpha": 25.0},
           mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0, "alpha": 2.0})
from ggs.mask import compute_importance_mask, prepare_target
from ggs import api
t = prepare_target(target, H, W)
m = compute_importance_mask(t, H, W, smooth=3, strength=0.7)
ev = {"s": 0.0}


def evaluate(G):
    t0 = time.perf_counter()
    f = api.fitness(G, t, H, W, 3.0, weight_mask=m)
    ev["s"] += time.perf_counter() - t0
    return f


if a.warm:                       # late-run regime: start from an annealed state
    init, _ = A.simulated_annealing(
        target, H, W, "cuda", a.splats, a.mutpb, cfg["mut_sigma_max"], cfg["mut_sigma_min"],
        "cosine", 3.0, 0.1, 3.0, 0.7, False, a.warm, 1e-3, "cosine", a.tries, seed=9,
        init_individual=init, progress=False, backend="device")
res = {}
variants = (("host_sequential", 1, "host", False, "host"),
            ("host_speculative", None, "host", False, "host"),
            ("device_host_loop", None, "device", False, "host"),
            ("device_loop_full", None, "device", False, "device"),
            ("device_loop_incremental", None, "device", True, "device"))
for name, spec, backend, inc, loop in variants:
    if a.only and name not in a.only.split(","):
        continue
    run = lambda n: A.simulated_annealing(          # noqa: E731
        target, H, W, "cuda", a.splats, a.mutpb, cfg["mut_sigma_max"], cfg["mut_sigma_min"],
        "cosine", 3.0, 0.1, 3.0, 0.7, False, n, a.temp0, "cosine", a.tries, seed=2,
        init_individual=init, evaluate=evaluate if backend == "host" else None, progress=False,
        return_state=True, speculate=(a.speculate or None) if backend == "device" else spec,
        backend=backend, incremental=inc, loop=loop)
    iters = a.dev_iters if loop == "device" else a.iters
    reps = a.repeat if loop == "device" else 1
    run(2)                                           # warm-up
    rates = []
    for _ in range(reps):
        ev["s"] = 0.0
        t0 = time.perf_counter()
        best, fit, st = run(iters)
        t_setup = time.perf_counter() - t0 - st["stats"]["loop_s"]
        rates.append(iters / st["stats"]["loop_s"])
    dt = iters / sorted(rates)[len(rates) // 2]
    res[name] = {"iters_per_s": round(iters / dt, 2), "ms_per_iter": round(dt / iters * 1e3, 2),
                 "iters": iters, "runs_iters_per_s": [round(r, 1) for r in rates],
                 "setup_ms": round(t_setup * 1e3, 1), "accepted": st["stats"].get("accepted"),
                 "eval_ms_per_iter": round(ev["s"] / a.iters * 1e3, 2) if backend == "host" else None,
                 "launches": st["stats"]["launches"], "evaluated": st["stats"]["evaluated"],
                 # trajectory-independent rates (the it/s of one seed depend on its acceptances)
                 "us_per_round": round(dt * 1e6 / max(1, st["stats"]["launches"]), 1),
                 "us_per_evaluated": round(dt * 1e6 / max(1, st["stats"]["evaluated"]), 1),
                 "changed_splats_per_neighbour": round(st["stats"]["changed_splats"] /
                                                       max(1, st["stats"]["proposed"]), 1)
                 if "changed_splats" in st["stats"] else None,
                 "best_fit": fit}
def same(x, y):
    if x in res and y in res and res[x]["iters"] == res[y]["iters"]:
        assert res[x]["best_fit"] == res[y]["best_fit"], (x, y)


same("host_sequential", "host_speculative")
same("device_host_loop", "device_loop_full")
same("device_loop_full", "device_loop_incremental")
print(json.dumps({"metric": "SA iterations/s", "config": {"H": H, "W": W, "splats": a.splats,
                  "tries_per_iter": a.tries, "mutpb": a.mutpb, "iters": a.iters, "temp0": a.temp0,
                  "warm_iters": a.warm}, **res}))
