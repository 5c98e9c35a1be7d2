"""Per-wave timing of one raster launch at any canvas / splat count / batch
(diagnostic build GGS_TIMING=1), through the host API.

    make -C genetic-gaussian-splats_amd/csrc probe PROBE=-DGGS_TIMING=1
    GGS_PROBE=1 GGS_LIB=genetic-gaussian-splats_amd/libggs_probe.so python tools/probe/wave_timing_cfg.py --size 2048 --splats 4096 --batch 1

Prints the launch span, the wave-duration spread, visits per wave, and the grid
fill: how long at least 3,072 / 2,048 / 1,024 waves were live."""
import argparse, ctypes as C, json, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "genetic-gaussian-splats_amd"))
import ggs
from ggs import ga

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=2048)
ap.add_argument("--splats", type=int, default=4096)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--dump", default="", help="save the raw per-wave records (npz) and print the longest waves")
a = ap.parse_args()
H = W = a.size
rng = np.random.default_rng(0)
tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
mask = rng.uniform(0.405, 1, (H, W)).astype(np.float32)
pop = ga.new_population(a.batch, a.splats, H, W, 3.0, 0.1, np.random.default_rng(a.batch))
for _ in range(3):
    ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
n_waves = a.batch * (-(-W // 64)) * (-(-H // 128)) * 4
buf = np.zeros((n_waves, 8), np.uint64)
fn = ggs.lib.ggs_debug_timing_read
fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_size_t]
assert fn(buf.ctypes.data, buf.nbytes) == 0, "not a GGS_TIMING build?"
def slot_gaps(buf, s_us, e_us):
    """Idle time between consecutive waves of one wave slot: HW_ID's wave / SIMD /
    CU / SH / SE fields (bits 0-15) + XCC_ID name the slot; the gap is the next
    wave's start minus this wave's end.  frac = the gaps over (slots x span)."""
    key = ((buf[:, 5] & np.uint64(0xFFFF)) | ((buf[:, 5] >> np.uint64(32) & np.uint64(0xF)) << np.uint64(16))).astype(np.int64)
    gaps, slots = [], 0
    for k in np.unique(key):
        i = np.where(key == k)[0]
        i = i[np.argsort(s_us[i])]
        slots += 1
        if len(i) > 1:
            gaps.extend((s_us[i[1:]] - e_us[i[:-1]]).tolist())
    g = np.asarray(gaps) if gaps else np.zeros(1)
    span = float(e_us.max())
    return {"slots": slots, "waves_per_slot": round(len(s_us) / max(slots, 1), 2),
            "gap_us": {q: round(float(np.percentile(g, p)), 3) for q, p in (("p10", 10), ("p50", 50), ("p90", 90))},
            "gap_us_mean": round(float(g.mean()), 3), "gaps_frac_of_slot_time": round(float(g.sum()) / (slots * span), 4)}


rt0, rt1 = buf[:, 0].astype(np.int64), buf[:, 1].astype(np.int64)
t0 = rt0.min()
s_us, e_us = (rt0 - t0) / 100.0, (rt1 - t0) / 100.0
dur = e_us - s_us
visits = buf[:, 6].astype(np.int64)
ts = np.linspace(0, e_us.max(), 400)
live = np.array([((s_us <= t) & (e_us > t)).sum() for t in ts])
dt = ts[1] - ts[0]
xcc = (buf[:, 5] >> np.uint64(32)).astype(np.int64) & 0xF
per_xcd_live = np.array([[((s_us <= t) & (e_us > t) & (xcc == x)).sum() for x in range(8)] for t in ts])
mid = (ts > 0.2 * ts[-1]) & (ts < 0.7 * ts[-1])
res = {"H": H, "splats": a.splats, "batch": a.batch, "waves": n_waves, "span_us": float(e_us.max()),
       "wave_us": {k: float(np.percentile(dur, q)) for k, q in (("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))},
       "wave_us_mean": float(dur.mean()),
       "visits": {k: int(np.percentile(visits, q)) for k, q in (("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))},
       "us_with_live_ge": {str(n): float((live >= n).sum() * dt) for n in (3072, 2048, 1024, 512)},
       "mean_live": float(live.mean()),
       "phase_frac": {k: round(float(buf[:, i].astype(np.float64).sum() / buf[:, 2:5].astype(np.float64).sum()), 3)
                      for k, i in (("cull", 2), ("visits", 3), ("epilogue", 4))},
       "blended": {k: int(np.percentile(buf[:, 7].astype(np.int64), q)) for k, q in (("p50", 50), ("max", 100))},
       "clk_per_blended_visit_p50": float(np.median(buf[:, 3].astype(np.float64) /
                                                    np.maximum(buf[:, 7].astype(np.float64), 1))),
       "ns_per_blended_visit_p50": float(np.median(dur * 1e3 / np.maximum(buf[:, 7].astype(np.float64), 1))),
       "last_start_us": float(s_us.max()),
       "xcd_work_ms": [round(float(dur[xcc == x].sum()) / 1e3, 2) for x in range(8)],
       "xcd_end_us": [round(float(e_us[xcc == x].max()), 1) for x in range(8)],
       "xcd_live_mid_mean": [round(float(per_xcd_live[mid, x].mean()), 1) for x in range(8)],
       "slot_gaps": slot_gaps(buf, s_us, e_us),
       "xcd_live_mid_max": [int(per_xcd_live[mid, x].max()) for x in range(8)],
       "xcd_full_frac_mid": float((per_xcd_live[mid] >= 384).any(axis=1).mean())}
print(json.dumps(res))
if a.dump:
    np.savez(a.dump, buf=buf)
    top = np.argsort(-dur)[:16]
    for w in top:     # block, us, cull/visit/epilogue clocks (100 MHz-independent s_memtime), listed, blended
        print("wave %6d  %6.1f us  cull %8d  visits %8d  epi %6d  listed %4d  blended %4d" %
              (w, dur[w], buf[w, 2], buf[w, 3], buf[w, 4], buf[w, 6], buf[w, 7]))
    q = np.argsort(dur)
    for lo, hi in ((0, 0.5), (0.5, 0.9), (0.9, 0.99), (0.99, 1.0)):
        sel = q[int(lo * len(q)):int(hi * len(q))]
        print("duration quantile %.2f-%.2f: mean %.1f us, listed %.0f, blended %.0f, cull share %.3f" %
              (lo, hi, dur[sel].mean(), buf[sel, 6].mean(), buf[sel, 7].mean(),
               buf[sel, 2].astype(float).sum() / buf[sel, 2:5].astype(float).sum()))
