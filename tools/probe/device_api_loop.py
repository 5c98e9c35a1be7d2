"""ggs_fitness_device in a loop (the drop-in's torch-on-GPU path: the target plan
is rebuilt on every call) at 512^2/256/128 — for a rocprofv3 kernel trace of
plan_kernel / plan_wsum_kernel next to prep / raster / finalize."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "genetic-gaussian-splats_amd"))
import ggs
from ggs import hip, ga
H = W = 512
rng = np.random.default_rng(0)
pop = hip.DeviceArray.from_host(ga.new_population(128, 256, H, W, 3.0, 0.1, rng))
tgt = hip.DeviceArray.from_host(rng.uniform(0, 1, (H, W, 3)).astype(np.float32))
mask = hip.DeviceArray.from_host(rng.uniform(0.4, 1, (H, W)).astype(np.float32))
out = hip.DeviceArray((128,))
st = hip.Stream()
for _ in range(5):
    ggs.fitness_device(0, st.handle, pop.ptr, 128, 256, 9, tgt.ptr, mask.ptr, ggs.GGS_FIT_WEIGHTED, 1.0, H, W,
                       3.0, out.ptr)
st.synchronize()
n, t0 = 200, time.perf_counter()
for _ in range(n):
    ggs.fitness_device(0, st.handle, pop.ptr, 128, 256, 9, tgt.ptr, mask.ptr, ggs.GGS_FIT_WEIGHTED, 1.0, H, W,
                       3.0, out.ptr)
st.synchronize()
print(f"device API (plan rebuilt per call): {(time.perf_counter() - t0) / n * 1e3:.4f} ms per call of 128")
