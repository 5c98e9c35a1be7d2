"""Per-workgroup phase clocks of the GA's variation / breed kernel (diagnostic
build GGS_VTIMING=1; thread 0's s_memrealtime, 100 MHz, at each phase boundary).

    make -C genetic-gaussian-splats_amd/csrc probe PROBE="-DGGS_TIMING=1 -DGGS_VTIMING=1"
    GGS_PROBE=1 GGS_LIB=genetic-gaussian-splats_amd/libggs_probe.so [P=32 N=512] python tools/probe/breed_timing.py

Runs 30 device-GA generations at the bench workload (512^2, 256 splats, pop 128)
and prints, for the last launch, the median/max time of each phase over the
workgroups (N <= 256 path): 0->1 phase A (row-map and gather loads, tournament
candidates, every per-splat draw), 1->2 tournament compare + any() barrier,
2->3 fallbacks, 3->4 parent row + mutation + size, 4->5 swap, 5->6 store + prep
+ gather store, and the kernel's first-start to last-end span.
Measured (512^2/256/128, fused breed): 5.16 / 0.68 / 0.48 / 1.00 / 0.72 / 2.58 us,
span 11.3 us (the kernel trace's 13.7 us includes launch)."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "genetic-gaussian-splats_amd"))
from ggs import ga, _lib                                            # noqa: E402
from ggs.ga_device import DeviceGA                                  # noqa: E402
from ggs.mask import compute_importance_mask, prepare_target        # noqa: E402

H = W = 512
P, N = int(os.environ.get("P", "128")), int(os.environ.get("N", "256"))
target = np.random.default_rng(0).uniform(0, 255, (H, W, 3)).astype(np.float32)
t = prepare_target(target, H, W)
m = compute_importance_mask(t, H, W, smooth=3, strength=0.7)
init = ga.new_population(P, N, H, W, 3.0, 0.1, np.random.default_rng(0))
cfg = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0, "alpha": 25.0},
           mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0, "alpha": 2.0},
           schedule="cosine")
dga = DeviceGA(t, m, init, tour_k=2, elite_k=8, cxpb=0.05, mutpb=0.05, min_scale_splats=3.0,
               max_scale_splats=0.1, seed=1, **cfg)
dga.run(1, 30, 30)
dga.read()
buf = np.zeros(8 * 4096, np.uint64)
lib = _lib.lib
lib.ggs_debug_vtiming_read.argtypes = [C.c_void_p, C.c_size_t]
assert lib.ggs_debug_vtiming_read(buf.ctypes.data, buf.nbytes) == 0
tm = buf.reshape(4096, 8)[:P].astype(np.int64)
names = ["phase A", "tournament", "fallbacks", "mutate", "swap", "store+prep"]
for k, nm in enumerate(names):
    d = (tm[:, k + 1] - tm[:, k]) * 10e-3   # us
    print(f"{nm:12s} median {np.median(d):7.2f} us  max {d.max():7.2f} us")
print(f"span {(tm[:, 6].max() - tm[:, 0].min()) * 10e-3:.2f} us; start spread {(tm[:, 0].max() - tm[:, 0].min()) * 10e-3:.2f} us")
dga.close()
