"""Breed kernel with the per-splat draws read from memory (the replay path) vs
computed by Philox, at the shipped GA shape (512², 512 splats, pop 32, elite 8):
the upper bound of precomputing the draws off the critical path.

    rocprofv3 --kernel-trace --stats -d gpurun_out/bd_<mode> -o run -- python3 tools/probe/breed_draws_ab.py --mode draws|philox
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "genetic-gaussian-splats_amd"), os.path.join(REPO, "tests")]
from ggs import ga  # noqa: E402
from ggs.ga_device import RecordingDraws  # noqa: E402
from ggs.mask import compute_importance_mask, prepare_target  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", choices=("draws", "philox"), required=True)
ap.add_argument("--gens", type=int, default=60)
a = ap.parse_args()
H = W = 512
P, N = 32, 512
CFG = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0, "alpha": 25.0},
           mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0, "alpha": 2.0},
           schedule="cosine")
target = np.random.default_rng(0).uniform(0, 255, (H, W, 3)).astype(np.float32)
init = ga.new_population(P, N, H, W, 3.0, 0.1, np.random.default_rng(1))
kw = dict(pop_size=P, n_splats=N, generations=a.gens, tour_k=3, elite_k=8, cxpb=0.9, mutpb=0.05,
          min_scale_splats=3.0, max_scale_splats=0.1, k_sigma=3.0, mask_strength=0.7, boost_only=False,
          init_population=init, progress=False, return_state=True, **CFG)
if a.mode == "draws":
    rec = RecordingDraws(ga.NumpyDraws(5), 0.9)
    ga.genetic_approx(target, H, W, "cuda", draws=rec, **kw)          # host GA records the draws
    ga.genetic_approx(target, H, W, "cuda", draws=rec, backend="device", chunk=a.gens, **kw)
else:
    ga.genetic_approx(target, H, W, "cuda", backend="device", chunk=a.gens, **kw)
print("done", a.mode)
