"""Golden fixture of the HEADLINE config (BASELINE.json configs[1]: 512x512 canvas,
256 splats) made by running the REFERENCE itself -> tests/golden/headline_512.npz.

Build container only (refuses without /root/reference), same method as
make_golden.py: the reference's modules are imported read-only and called by
name; its Triton kernel ``_render_tile_over_kernel`` runs under the Triton
interpreter (``TRITON_INTERPRET=1``) through make_golden.ref_render_cpu, which
sequences render.py:226-252 on the CPU.

Stored: one candidate in the GA's axes-angle layout (population.py:20-46
distributions), its renderer genome (encode.py), the image the reference renders
at tile 64 (render.py:210, render_splats_rgb_triton's default) over the whole
canvas, an 8-bit target (stored as uint8; the float target is u8 / 255), the
reference's importance mask of that target (mask.py, algorithm.py:42-49
arguments) and the reference's fitness_many scalars in the three modes at the
GA's tile 32 (fitness.py:7-31).

    python tests/golden/make_golden_512.py      (~1-2 min under the interpreter)
"""
from __future__ import annotations

import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (sets TRITON_INTERPRET, imports the reference)

import numpy as np  # noqa: E402

E, F, M, t, CPU = MG.E, MG.F, MG.M, MG.t, MG.CPU


def main() -> None:
    H = W = 512
    N = 256
    pop = MG.synthetic_population(1, N, H, W, seed=512)               # [1, 256, 9] axes layout
    g9 = E.genome_to_renderer_batched(t(pop)).numpy()
    t0 = time.time()
    img64 = MG.ref_render_cpu(t(g9), H, W, k_sigma=3.0, tile=64).numpy()
    print(f"render tile 64: {time.time() - t0:.1f} s")
    rng = np.random.default_rng(512)
    target_u8 = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)      # an 8-bit image, /255 as
    target = target_u8.astype(np.float32) / np.float32(255.0)       # algorithm.py:33-39 does
    mask = M.compute_importance_mask(t(target), H, W, edge_scales=(1, 2, 4), w_edge=0.7, w_var=0.3,
                                     gamma=0.7, floor=0.15, smooth=3, strength=0.7).numpy()
    F.render_splats_rgb_triton = MG.ref_render_cpu      # fitness.py:4 imports the name
    plist = [t(p) for p in pop]
    fit = {}
    for mode, kw in (("none", {}), ("weighted", {"weight_mask": t(mask)}),
                     ("boost", {"weight_mask": t(mask), "boost_only": True})):
        t0 = time.time()
        fit[mode] = F.fitness_many(plist, t(target), H, W, 3.0, CPU, **kw).numpy()
        print(f"fitness {mode}: {fit[mode]} ({time.time() - t0:.1f} s)")
    np.savez_compressed(os.path.join(HERE, "headline_512.npz"), pop=pop, genomes=g9, img_t64=img64,
                        target_u8=target_u8, mask=mask, HWk=np.array([H, W, 3.0], np.float64),
                        **{f"fit_{k}": v for k, v in fit.items()})
    print("done")


if __name__ == "__main__":
    main()
