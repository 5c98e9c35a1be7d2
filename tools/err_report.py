"""Max |GPU - oracle| image error at the BASELINE configurations (crops of the
large ones), for the parity margin against the 1e-4 bar.
usage: python tools/err_report.py"""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genetic-gaussian-splats_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ggs
import ggs_oracle as O

out = {}
for (H, N, B, seed) in ((128, 32, 8, 0), (512, 256, 4, 1), (1024, 1024, 2, 2), (2048, 4096, 1, 3)):
    pop = O.synthetic_population(B, N, H, H, seed=seed)
    g9 = O.genome_to_renderer_batched(pop)
    img = ggs.render(ggs.encode(pop), H, H)
    wins = [(0, H, 0, H)] if H <= 512 else [(H // 2 - 64, H // 2 + 64, H // 2 - 64, H // 2 + 64),
                                          (0, 96, 0, 96), (H - 96, H, H // 3, H // 3 + 96)]
    errs = []
    for b in range(B):
        for (y0, y1, x0, x1) in wins:
            ref = O.render(g9[b:b + 1], H, H, window=(y0, y1, x0, x1))[0]
            errs.append(float(np.abs(img[b, y0:y1, x0:x1] - ref).max()))
    out[f"{H}x{H}/{N}"] = {"max_abs_err": max(errs), "mean_of_max": float(np.mean(errs))}
print(json.dumps(out))
