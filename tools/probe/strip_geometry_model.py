"""Model of raster work per candidate for strip widths 8-64 (VALU ~30 per visit + 7 per
pair step), over the bench population: visits, pair steps, pairs per visit."""
import sys, numpy as np
import os
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'oracle')]
import bench, ggs_oracle as O
def model(size, N, B, SW, head=30, pk=7):
    bench.H = bench.W = size
    pop = bench.synthetic_population(B, N, 10_000)
    P = 64 // SW; SH = 32 * P
    V = S = 0
    for b in range(B):
        p = O.preprocess(O.genome_to_renderer_batched(pop[b][None])[0], size, size, 3.0)
        x0, x1, y0, y1 = (p[k].astype(np.int64) for k in ("x0", "x1", "y0", "y1"))
        for i in range(N):
            for ty in range(y0[i] // SH, y1[i] // SH + 1):
                ty0 = ty * SH
                a = (max(y0[i], ty0) - ty0) // (2 * P); c = (min(y1[i], ty0 + SH - 1) - ty0) // (2 * P)
                ns = x1[i] // SW - x0[i] // SW + 1
                V += ns; S += ns * (c - a + 1)
    return V / B, S / B, (V * head + S * pk) / B
for size, N in ((512, 256), (1024, 1024)):
    for SW in (8, 16, 32, 64):
        v, s, c = model(size, N, 4, SW)
        print(size, N, 'SW', SW, 'visits/cand %.0f pairsteps/cand %.0f pairs/visit %.2f VALU/cand %.0f' % (v, s, s / v, c))
