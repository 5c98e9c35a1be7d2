"""Per-wave timing of the device GA's raster at the shipped shape (512^2, 512
splats, 24 evaluated) with and without the single-round packing (GGS_GA_LPT),
from the GGS_TIMING probe build:

    make -C genetic-gaussian-splats_amd/csrc probe PROBE=-DGGS_TIMING=1
    GGS_PROBE=1 GGS_LIB=$PWD/genetic-gaussian-splats_amd/libggs_probe.so GGS_GA_LPT=1 python tools/probe/lpt_waves.py

The timing buffer holds the last raster launch of the run (indexed by block).
Prints: the launch span, whether the waves sharing a SIMD are blocks r, r + S,
r + 2S, the per-SIMD sums of blended visits (max / median), the correlation of a
SIMD's end time with that sum and with its longest wave, and what the last wave
to end was doing."""
import ctypes as C, json, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "genetic-gaussian-splats_amd"))
import ggs
from ggs import ga
from ggs.ga_device import DeviceGA
from ggs.mask import compute_importance_mask, prepare_target

H = W = 512
P, N, E = 32, 512, 8
gens = int(os.environ.get("GENS", "60"))
target = np.random.default_rng(0).uniform(0, 255, (H, W, 3)).astype(np.float32)
t = prepare_target(target, H, W)
m = compute_importance_mask(t, H, W, smooth=3, strength=0.7)
init = ga.new_population(P, N, H, W, 3.0, 0.1, np.random.default_rng(0))
cfg = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0, "alpha": 25.0},
           mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0, "alpha": 2.0},
           schedule="cosine")
dga = DeviceGA(t, m, init, tour_k=2, elite_k=E, cxpb=0.05, mutpb=0.05, min_scale_splats=3.0,
               max_scale_splats=0.1, seed=1, **cfg)
dga.run(1, gens, gens)
st = dga.read()
n = (P - E) * 128
buf = np.zeros((n, 8), np.uint64)
fn = ggs.lib.ggs_debug_timing_read
fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_size_t]
assert fn(buf.ctypes.data, buf.nbytes) == 0, "not a GGS_TIMING build?"
rt0, rt1 = buf[:, 0].astype(np.int64), buf[:, 1].astype(np.int64)
t0 = rt0.min()
s_us, e_us = (rt0 - t0) / 100.0, (rt1 - t0) / 100.0
hw = buf[:, 5]
# SIMD key: HW_ID's SIMD (bits 4-5), CU (8-11), SH (12), SE (13-15) + XCC_ID
key = (((hw >> np.uint64(4)) & np.uint64(0x3)) | (((hw >> np.uint64(8)) & np.uint64(0xFF)) << np.uint64(2)) |
       (((hw >> np.uint64(32)) & np.uint64(0xF)) << np.uint64(10))).astype(np.int64)
done = buf[:, 7].astype(np.int64)
S = 1024
grp_ok = 0
simds = {}
for b in range(n):
    simds.setdefault(int(key[b]), []).append(b)
for k, bl in simds.items():
    bl = sorted(bl)
    if len(bl) >= 2 and all((x - bl[0]) % S == 0 for x in bl):
        grp_ok += 1
ends = np.array([e_us[bl].max() for bl in simds.values()])
sums = np.array([done[bl].sum() for bl in simds.values()])
longest = np.array([(e_us[bl] - s_us[bl]).max() for bl in simds.values()])
last = int(np.argmax(e_us))
lk = int(key[last])
mates = sorted(simds[lk])
res = {"lpt": os.environ.get("GGS_GA_LPT", "1"), "gens": gens, "best_fit": st["best_fit"],
       "span_us": round(float(e_us.max()), 2), "waves": n, "simds_seen": len(simds),
       "simds_grouped_r_rS_r2S": grp_ok,
       "simd_visit_sum": {"max": int(sums.max()), "p50": int(np.median(sums)), "mean": round(float(sums.mean()), 1)},
       "corr_end_vs_sum": round(float(np.corrcoef(ends, sums)[0, 1]), 3),
       "corr_end_vs_longest_wave": round(float(np.corrcoef(ends, longest)[0, 1]), 3),
       "wave_us": {"p50": round(float(np.median(e_us - s_us)), 2), "max": round(float((e_us - s_us).max()), 2)},
       "last_wave": {"block": last, "start_us": round(float(s_us[last]), 2), "end_us": round(float(e_us[last]), 2),
                     "blended": int(done[last]),
                     "simd_mates": [{"block": b, "blended": int(done[b]), "end_us": round(float(e_us[b]), 2)}
                                    for b in mates]},
       "top_simd_sums": sorted(sums.tolist())[-5:],
       "blended_max": int(done.max()), "blended_p50": int(np.median(done))}
print(json.dumps(res))
