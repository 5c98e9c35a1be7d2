"""Probe: does torch's HIP runtime initialise after libggs created sessions?"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "genetic-gaussian-splats_amd"))
import numpy as np
import ggs
from ggs import ga
from ggs.ga_device import DeviceSA
mode = sys.argv[1]
H = W = 32
t = np.random.default_rng(0).uniform(0, 1, (H, W, 3)).astype(np.float32)
m = np.ones((H, W), np.float32)
cfg = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0, "alpha": 25.0},
           mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0, "alpha": 2.0})
if mode == "torch_first":
    import torch
    print("torch first:", torch.cuda.is_available(), torch.zeros(1).cuda())
n = int(sys.argv[2]) if len(sys.argv) > 2 else 0
print("fitness", ggs.fitness(ga.new_population(2, 4, H, W, 3, 0.1), t, H, W, 3.0, weight_mask=m))
for i in range(n):
    sa = DeviceSA(t, m, ga.new_population(1, 4, H, W, 3, 0.1)[0], max_tries=2, mutpb=0.1,
                  schedule="cosine", min_scale_splats=3, max_scale_splats=0.1, **cfg)
    sa.propose(0, 1, 0, 2)
    sa.close()
import torch
print("torch after", n, "sessions:", torch.cuda.is_available(), torch.cuda.device_count())
print(torch.zeros(1).cuda())
