"""The render API (render_splats_rgb_triton, render.py:203-252) on the device
path: ggs_render_device = prep (no encode) + raster_kernel<0, *, false> writing
[B, H, W, 3] float32 clamped images to HBM.

Presets (--preset):
  batch   512x512, 256 splats, B 128 (the bench population rendered as images)
  frame   512x512, 512 splats, B 1 (save_frame_png, utils.py:48-69: the GA's
          snapshot of its best individual at the work size)
  final   2048x1536, 512 splats, B 1 (run_ggs.py:64-72: the best genome rescaled
          to the full-resolution target, resize.py:16-20, rendered once; a 4:3
          photo whose work size is 512x384)

Reports renders/s and ms per launch (HIP events around the raster alone and a
host-timed loop of the whole call), and the algorithmic bytes per candidate
12*H*W (image written) + 36*N (genome read) against 8 TB/s.  Under
tools/profile.sh (BENCH="python3 tools/bench_render.py ...") the PMC passes give
the raster's WRITE_SIZE against 12*H*W*B.

usage: python tools/bench_render.py [--preset batch|frame|final] [--iters 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "genetic-gaussian-splats_amd"), REPO]
os.environ.setdefault("GGS_HIP_RUNTIME", "system")
import bench  # noqa: E402  (synthetic population: population.py distributions)
import ggs  # noqa: E402
from ggs import hip  # noqa: E402

PRESETS = {"batch": dict(H=512, W=512, splats=256, B=128, scale=1.0),
           "frame": dict(H=512, W=512, splats=512, B=1, scale=1.0),
           "final": dict(H=1536, W=2048, splats=512, B=1, scale=4.0)}

ap = argparse.ArgumentParser()
ap.add_argument("--preset", default="batch", choices=sorted(PRESETS))
ap.add_argument("--iters", type=int, default=200)
ap.add_argument("--min-time", type=float, default=0.5)
a = ap.parse_args()
p = PRESETS[a.preset]
H, W, N, B = p["H"], p["W"], p["splats"], p["B"]

# work-size genomes (max side 512), then resize.py:16-20's log-scale shift to the
# output size (x, y stay normalised), then encode -> renderer layout
wH, wW = int(round(H / p["scale"])), int(round(W / p["scale"]))
bench.H, bench.W = wH, wW
G = bench.synthetic_population(B, N, 7)
if p["scale"] != 1.0:
    G[..., 2] += np.float32(np.log(W / wW))
    G[..., 3] += np.float32(np.log(H / wH))
R = ggs.encode(G)

ggs.ensure_init()
hip.set_device(0)
st = hip.Stream()
g = hip.DeviceArray.from_host(np.ascontiguousarray(R, np.float32))
out = hip.DeviceArray((B, H, W, 3))


def call():
    ggs.render_device(0, st.handle, g.ptr, B, N, 9, H, W, 3.0, out.ptr)


for _ in range(10):                               # warm-up + clocks
    call()
st.synchronize()
t0, n = time.perf_counter(), 0
while time.perf_counter() - t0 < a.min_time or n < a.iters:
    call()
    n += 1
st.synchronize()
dt = (time.perf_counter() - t0) / n
ggs.profile_reset()
ggs.profile_enable(True)
for _ in range(min(a.iters, 100)):
    call()
st.synchronize()
ggs.profile_enable(False)
kern = {k: ggs.profile_read(k) for k in ("prep", "raster")}
raster_ms = kern["raster"][0] / max(kern["raster"][1], 1)
alg = 12 * H * W + 36 * N
# parity spot check against nothing external: the image is finite and in [0, 1]
img = out.to_host()
assert np.isfinite(img).all() and img.min() >= 0 and img.max() <= 1
print(json.dumps({
    "preset": a.preset, "H": H, "W": W, "splats": N, "B": B,
    "renders_per_s": round(B / dt, 1), "ms_per_call": round(dt * 1e3, 4),
    "kernels_ms_per_launch": {k: round(v[0] / max(v[1], 1), 5) for k, v in kern.items()},
    "algorithmic_bytes_per_candidate": alg,
    "raster_achieved_GBps": round(alg * B / (raster_ms * 1e-3) / 1e9, 1),
    "raster_hbm_frac": round(alg * B / (raster_ms * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 4),
    "image_bytes_per_launch": 12 * H * W * B,
}))
