"""Host render API (ggs.render on numpy arrays) per call: a GA frame (512², 512
splats, B 1), the final full-res render (2048x1536, 512 splats) and a 512²/256/8 batch."""
import os, sys, time
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                             "genetic-gaussian-splats_amd")]
import ggs
from ggs import ga
for (H, W, N, B) in ((512, 512, 512, 1), (1536, 2048, 512, 1), (512, 512, 256, 8)):
    pop = ga.new_population(B, N, H, W, 3.0, 0.1, np.random.default_rng(1))
    g = ggs.encode(pop)
    for _ in range(5):
        ggs.render(g, H, W)
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < 0.5:
        img = ggs.render(g, H, W)
        n += 1
    print(f"render {H}x{W} N={N} B={B}: {(time.perf_counter() - t0) / n * 1e3:.3f} ms per call, checksum {float(img.sum()):.4f}")
