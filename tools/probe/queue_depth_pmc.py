"""Probe: does rocprofv3 --pmc survive K fitness evaluations (3 dispatches each)
enqueued behind ONE host sync?  Tiny workload (64^2, 8 splats, 4 candidates), so
only the number of queued dispatches varies.  Used to establish the cause of the
round-2 SIGSEGV in ggs_sa_run under --pmc (docs/EXPERIMENTS.md §9).

    rocprofv3 --pmc FETCH_SIZE -- python3 tools/probe/queue_depth_pmc.py K
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "genetic-gaussian-splats_amd"))
os.environ.setdefault("GGS_HIP_RUNTIME", "system")
import ggs  # noqa: E402
from ggs import hip  # noqa: E402

K = int(sys.argv[1])
H = W = 64
B, N = 4, 8
ggs.ensure_init()
hip.set_device(0)
rng = np.random.default_rng(0)
G = np.concatenate([rng.uniform(0, 1, (B, N, 2)), rng.uniform(1, 2, (B, N, 2)), rng.uniform(-3, 3, (B, N, 1)),
                    rng.uniform(0, 255, (B, N, 4))], -1).astype(np.float32)
g = hip.DeviceArray.from_host(G)
t = hip.DeviceArray.from_host(rng.uniform(0, 1, (H, W, 3)).astype(np.float32))
m = hip.DeviceArray.from_host(rng.uniform(0.4, 1, (H, W)).astype(np.float32))
out = hip.DeviceArray((B,))
st = hip.Stream()
plan = ggs.TargetPlan(0, st.handle, t.ptr, m.ptr, ggs.GGS_FIT_WEIGHTED, 1.0, H, W)
st.synchronize()
for _ in range(K):
    plan.fitness_device(st.handle, g.ptr, B, N, 9, 3.0, out.ptr)
st.synchronize()
print(f"queue_depth_pmc: {K} evaluations ({3 * K} dispatches) behind one sync: ok", flush=True)
