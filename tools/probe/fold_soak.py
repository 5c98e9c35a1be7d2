"""Soak of the finalize folded into the raster (device GA): a long run of the
shipped GA shape (config.py: 512^2, 512 splats, pop 32, elite 8) — or the bench
shape (SOAK_SHAPE=bench) — with Philox draws, printed as a digest of the final
population, fitness vector, best fitness and curves.  Run it twice, with and
without GGS_UNFUSED_FINALIZE=1: one stale partial read anywhere in the run
changes a fitness value and with it the whole later trajectory, so equal digests
over G generations mean every one of the G x (P - E) folded reductions read what
the separate finalize launch reads.

    [GGS_UNFUSED_FINALIZE=1] SOAK_GENS=100000 python tools/probe/fold_soak.py"""
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "genetic-gaussian-splats_amd"))
from ggs import ga                                                   # noqa: E402
from ggs.ga_device import DeviceGA                                   # noqa: E402
from ggs.mask import compute_importance_mask, prepare_target         # noqa: E402

CFG = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0, "alpha": 25.0},
           mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0, "alpha": 2.0},
           schedule="cosine")
P, N = (128, 256) if os.environ.get("SOAK_SHAPE") == "bench" else (32, 512)
H = W = 512
G = int(os.environ.get("SOAK_GENS", "20000"))
target = np.random.default_rng(0).uniform(0, 255, (H, W, 3)).astype(np.float32)
t = prepare_target(target, H, W)
m = compute_importance_mask(t, H, W, smooth=3, strength=0.7)
init = ga.new_population(P, N, H, W, 3.0, 0.1, np.random.default_rng(0))
dga = DeviceGA(t, m, init, tour_k=2, elite_k=8, cxpb=0.05, mutpb=0.05, min_scale_splats=3.0,
               max_scale_splats=0.1, seed=3, **CFG)
t0 = time.perf_counter()
for c in range(0, G, 5000):
    dga.run(1 + c, min(5000, G - c), G)
    print(f"  {min(G, c + 5000)} generations, {time.perf_counter() - t0:.1f} s", flush=True)
st = dga.read()
h = hashlib.sha256()
for a in (st["population"], st["fitness"], np.float64(st["best_fit"]),
          *(np.asarray(st["curves"][k]) for k in ("best", "mean", "median"))):
    h.update(np.ascontiguousarray(a).tobytes())
print(f"shape P={P} N={N} gens={G} unfused={os.environ.get('GGS_UNFUSED_FINALIZE', '0')} "
      f"best={st['best_fit']!r} digest={h.hexdigest()[:32]}")
dga.close()
