"""Model: how many raster pair steps land on 16x8 pixel blocks that are already
saturated (every pixel's transmittance below 2^-24) when the splat is blended?

A pair step of the raster is one splat on one 16-column x 8-row block of a strip
(lane (c, ph) rows 8k+ph and 8k+4+ph).  The kernel executes the pair steps of rows
[y0, y1] of every (splat, strip) visit; a block-level saturation skip would drop
the ones whose block is saturated.  Front-to-back over the population of bench.py.

    python tools/probe/pair_sat_model.py [--size 512] [--splats 256] [--cands 4]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
import bench  # noqa: E402
import ggs_oracle as O  # noqa: E402


def model(G, H, W, eps=2.0 ** -24):
    p = O.preprocess(O.genome_to_renderer_batched(G[None])[0], H, W, 3.0)
    N = G.shape[0]
    T = np.ones((H, W), np.float64)
    steps = skip = 0
    for i in range(N - 1, -1, -1):                      # front to back
        x0, x1, y0, y1 = (int(p[k][i]) for k in ("x0", "x1", "y0", "y1"))
        # blocks: 16-col strips x 8-row bands touched by the AABB
        bx0, bx1 = x0 // 16, x1 // 16
        by0, by1 = y0 // 8, y1 // 8
        for by in range(by0, by1 + 1):
            r0, r1 = by * 8, min(by * 8 + 8, H)
            tb = T[r0:r1, bx0 * 16:min((bx1 + 1) * 16, W)]
            for bx in range(bx0, bx1 + 1):
                steps += 1
                blk = tb[:, (bx - bx0) * 16:(bx - bx0) * 16 + 16]
                if blk.max() < eps:
                    skip += 1
        X = np.arange(x0, x1 + 1, dtype=np.float64)[None, :]
        Y = np.arange(y0, y1 + 1, dtype=np.float64)[:, None]
        qx, qy = X - p["cx"][i], Y - p["cy"][i]
        quad = p["sxx"][i] * qx * qx + 2 * p["sxy"][i] * qx * qy + p["syy"][i] * qy * qy
        f = np.exp(-0.5 * quad) * p["a"][i]
        T[y0:y1 + 1, x0:x1 + 1] *= 1.0 - f
    return steps, skip, T


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--splats", type=int, default=256)
    ap.add_argument("--cands", type=int, default=4)
    a = ap.parse_args()
    bench.H = bench.W = a.size
    pop = bench.synthetic_population(a.cands, a.splats, 10_000)
    tot = sk = 0
    for b in range(a.cands):
        s, k, T = model(pop[b], a.size, a.size)
        tot += s
        sk += k
        print(f"candidate {b}: {s} block steps, {k} on saturated blocks ({k / s:.1%}); "
              f"pixels with T < 2^-24 at the end: {(T < 2.0 ** -24).mean():.1%}", flush=True)
    print(f"total: {sk / tot:.1%} of block steps land on saturated blocks")


if __name__ == "__main__":
    main()
