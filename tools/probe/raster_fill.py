"""Raster time vs batch size (grid fill) at a given canvas / splat count, through
the host API with libggs's per-kernel event timing.  SA rounds at configs[4]
(2048^2, 4096 splats) evaluate 1-16 neighbours, 2,048 strip-waves each, against
3,072 wave slots.

usage: python tools/probe/raster_fill.py [--size 2048] [--splats 4096] [--batches 1,2,3,4,8,16]"""
import argparse, json, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "genetic-gaussian-splats_amd"))
import ggs
from ggs import ga

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=2048)
ap.add_argument("--splats", type=int, default=4096)
ap.add_argument("--batches", default="1,2,3,4,6,8,12,16")
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
H = W = a.size
rng = np.random.default_rng(0)
tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
mask = rng.uniform(0.405, 1, (H, W)).astype(np.float32)
out = {}
for B in [int(x) for x in a.batches.split(",")]:
    pop = ga.new_population(B, a.splats, H, W, 3.0, 0.1, np.random.default_rng(B))
    ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)          # warm (plan, buffers)
    ggs.profile_reset()
    ggs.profile_enable(True)
    for _ in range(a.reps):
        ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
    ggs.profile_enable(False)
    ms, n = ggs.profile_read("raster")
    out[B] = {"raster_ms": round(ms / max(n, 1), 4), "per_candidate_ms": round(ms / max(n, 1) / B, 4)}
print(json.dumps({"H": H, "splats": a.splats, "raster_by_batch": out}))
