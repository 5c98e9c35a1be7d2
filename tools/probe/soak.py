"""Longer device-GA and device-SA runs (Philox draws) checked for finite values,
in-range genomes and monotone best curves — insurance against rare numerical
paths (tiny Box-Muller radii, the recurrence guard, saturation cut-off)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "genetic-gaussian-splats_amd"))
from ggs import ga, annealing as A
from ggs.ga_device import DeviceGA
from ggs.mask import compute_importance_mask, prepare_target

CFG = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0, "alpha": 25.0},
           mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0, "alpha": 2.0},
           schedule="cosine")
H = W = 512
target = np.random.default_rng(0).uniform(0, 255, (H, W, 3)).astype(np.float32)
t = prepare_target(target, H, W)
m = compute_importance_mask(t, H, W, smooth=3, strength=0.7)
G = int(os.environ.get("SOAK_GENS", "5000"))
init = ga.new_population(128, 256, H, W, 3.0, 0.1, np.random.default_rng(0))
dga = DeviceGA(t, m, init, tour_k=2, elite_k=8, cxpb=0.05, mutpb=0.05, min_scale_splats=3.0,
               max_scale_splats=0.1, seed=7, **CFG)
t0 = time.perf_counter()
for c in range(0, G, 500):
    dga.run(1 + c, min(500, G - c), G)
    st = dga.read()
    P = st["population"]
    assert np.isfinite(P).all() and np.isfinite(st["fitness"]).all(), "non-finite GA state"
    lo, hi = ga.scale_log_bounds(H, W, 3.0, 0.1)
    assert (P[..., 0:2] >= 0).all() and (P[..., 0:2] <= 1).all()
    assert (P[..., 2:4] >= lo).all() and (P[..., 2:4] <= hi).all()
    assert (P[..., 5:9] >= 0).all() and (P[..., 5:9] <= 255).all()
    b = st["curves"]["best"]
    assert all(y <= x for x, y in zip(b, b[1:])), "best curve not monotone"
    print(f"GA gen {c + 500}: best {b[-1]:.6f} ({time.perf_counter() - t0:.1f} s)", flush=True)
dga.close()
HS = 2048
tgt2 = np.random.default_rng(1).uniform(0, 255, (HS, HS, 3)).astype(np.float32)
iters = int(os.environ.get("SOAK_SA_ITERS", "3000"))
best, fit, st = A.simulated_annealing(tgt2, HS, HS, "cuda", 4096, 0.05, CFG["mut_sigma_max"], CFG["mut_sigma_min"],
                                      "cosine", 3.0, 0.1, 3.0, 0.7, False, iters, 1e-3, "cosine", 8, seed=3,
                                      progress=False, return_state=True, backend="device")
cb, cc = st["curves"]["best"], st["curves"]["current"]
assert np.isfinite(best).all() and np.isfinite(cb).all() and np.isfinite(cc).all()
assert all(y <= x for x, y in zip(cb, cb[1:])), "SA best curve not monotone"
print(f"SA {iters} iterations at 2048^2/4096: best {fit:.6f}, accepted {st['stats'].get('accepted')}, "
      f"loop {st['stats']['loop_s']:.2f} s", flush=True)
print("soak ok")
