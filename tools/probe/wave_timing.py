"""Per-wave phase timing of the raster kernel (diagnostic build GGS_TIMING=1).

    make -C genetic-gaussian-splats_amd/csrc probe PROBE=-DGGS_TIMING=1
    GGS_PROBE=1 GGS_LIB=genetic-gaussian-splats_amd/libggs_probe.so python tools/probe/wave_timing.py

Runs the bench workload (512^2 / 256 splats / B = 128, weighted fitness), then
reads g_ggs_timing: per wave the realtime start/end (100 MHz), shader clocks
spent in cull / visits / epilogue, HW_ID/XCC_ID and visit count.  Prints the
phase split, the wave-duration spread, per-XCD end times and the occupancy
timeline (live waves vs. time, the grid's tail).
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "genetic-gaussian-splats_amd"))


def main():
    import torch
    import bench
    import ggs
    H = W = 512
    N, B = 256, int(os.environ.get("ABL_B", "128"))
    dev = torch.device("cuda", 0)
    g = torch.from_numpy(bench.synthetic_population(B, N, 0)).to(dev)
    rng = np.random.default_rng(1234)
    tgt = torch.from_numpy(rng.uniform(0, 1, (H, W, 3)).astype(np.float32)).to(dev)
    mask = torch.from_numpy(rng.uniform(0.405, 1, (H, W)).astype(np.float32)).to(dev)
    out = torch.empty(B, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    plan = ggs.TargetPlan(0, st, tgt.data_ptr(), mask.data_ptr(), 1, 1.0, H, W)
    for _ in range(5):
        plan.fitness_device(st, g.data_ptr(), B, N, 9, 3.0, out.data_ptr())
    torch.cuda.synchronize()
    n_waves = B * 32 * 4
    buf = np.zeros((n_waves, 8), np.uint64)
    fn = ggs.lib.ggs_debug_timing_read
    fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_size_t]
    assert fn(buf.ctypes.data, buf.nbytes) == 0, "ggs_debug_timing_read failed (not a GGS_TIMING build?)"
    rt0, rt1 = buf[:, 0].astype(np.int64), buf[:, 1].astype(np.int64)
    t0 = rt0.min()
    start_us, end_us = (rt0 - t0) / 100.0, (rt1 - t0) / 100.0     # 100 MHz realtime
    cull, vis, epi = (buf[:, k].astype(np.float64) for k in (2, 3, 4))
    tot = cull + vis + epi
    xcc = (buf[:, 5] >> np.uint64(32)).astype(np.int64) & 0xF
    visits = buf[:, 6].astype(np.int64)
    dur = end_us - start_us
    res = {
        "kernel_span_us": float(end_us.max()),
        "phase_frac": {"cull": float(cull.sum() / tot.sum()), "visits": float(vis.sum() / tot.sum()),
                       "epilogue": float(epi.sum() / tot.sum())},
        "shader_clk_per_wave": {"cull": float(cull.mean()), "visits": float(vis.mean()),
                                "epilogue": float(epi.mean())},
        "clk_per_visit": float(vis.sum() / max(visits.sum(), 1)),
        "visits_per_wave": float(visits.mean()),
        "wave_us": {"mean": float(dur.mean()), "p50": float(np.median(dur)), "p99": float(np.percentile(dur, 99)),
                    "max": float(dur.max())},
        "xcd_end_us": [float(end_us[xcc == x].max()) if (xcc == x).any() else None for x in range(8)],
    }
    # occupancy timeline: live waves per 2 us bin, and when the chip stops being full
    span = end_us.max()
    bins = np.arange(0, span + 2, 2.0)
    live = [int(((start_us <= b) & (end_us > b)).sum()) for b in bins]
    full = max(live)
    below = [b for b, l in zip(bins, live) if l < 0.9 * full and b > 5]
    res["live_waves_max"] = full
    res["tail_start_us"] = float(below[0]) if below else None
    res["live_timeline"] = live
    # wave-time-weighted idle: sum over bins of (full - live) * 2us / (full * span)
    res["slot_idle_frac"] = float(sum(full - l for l in live) * 2.0 / (full * span))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
