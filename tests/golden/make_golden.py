"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run in the build container only (``python tests/golden/make_golden.py``); it
refuses to run when /root/reference is absent (the GPU box).  It imports the
reference's own modules read-only (no bytecode is written) and calls them by
name; the only code here is input generation and a CPU driver that sequences
the reference's three render stages exactly as ``render_splats_rgb_triton``
does (render.py:226-252) on ``device='cpu'`` — that function itself asserts a
CUDA device (render.py:217), and the Triton kernel ``_render_tile_over_kernel``
runs under the Triton interpreter (``TRITON_INTERPRET=1``, numpy-backed).

Outputs (all small .npz, float32/int32, plus meta.json with library versions):
  encode.npz      encode.py genome_to_renderer_batched on edge-case genomes
  preprocess.npz  render.py _preprocess_genome outputs (13 arrays) per case
  render_*.npz    rendered images [B,H,W,3] per case (inputs included)
  fitness.npz     fitness.py fitness_many / fitness_population scalars
  mask.npz        mask.py compute_importance_mask on a synthetic target
"""
from __future__ import annotations

import json
import math
import os
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

if not os.path.isdir(os.path.join(REF, "modules")):
    raise SystemExit("make_golden.py: /root/reference is not present; fixtures are "
                     "generated in the build container only")

os.environ["TRITON_INTERPRET"] = "1"
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import triton  # noqa: E402

import modules.encode as E  # noqa: E402  (reference)
import modules.fitness as F  # noqa: E402  (reference)
import modules.mask as M  # noqa: E402  (reference)
import modules.render as R  # noqa: E402  (reference)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
from ggs_oracle import synthetic_population  # noqa: E402  (input spec only)

CPU = torch.device("cpu")


def ref_render_cpu(genomes: torch.Tensor, H: int, W: int, *, k_sigma: float = 3.0,
                   device=None, background=(1.0, 1.0, 1.0), tile: int = 32,
                   **_unused) -> torch.Tensor:
    """Sequence the reference's stages on CPU (mirrors render.py:219-252)."""
    g = genomes if genomes.ndim == 3 else genomes.unsqueeze(0)
    B, N, _ = g.shape
    parts = [R._preprocess_genome(g[b], H, W, k_sigma, CPU) for b in range(B)]
    cat = {key: torch.cat([p[key] for p in parts]) for key in parts[0]}
    flat_idx, tile_off, tile_cnt, nTX, _nTY, ntiles = R._gpu_bin_splats_to_tiles(
        cat["x0"], cat["x1"], cat["y0"], cat["y1"], B, N, H, W, tile)
    canvas = torch.empty((B, H, W, 3), dtype=torch.float32)
    canvas[:] = torch.as_tensor(background, dtype=torch.float32)
    sb, sh, sw, _ = canvas.stride()
    R._render_tile_over_kernel[(B * ntiles,)](
        canvas, H, W, sb, sh, sw,
        cat["cx"], cat["cy"], cat["sxx"], cat["sxy"], cat["syy"],
        cat["rc"], cat["gc"], cat["bc"], cat["a"],
        cat["x0"], cat["x1"], cat["y0"], cat["y1"],
        flat_idx, tile_off, tile_cnt, nTX, ntiles, TILE_W=tile, TILE_H=tile)
    return canvas.clamp_(0.0, 1.0)


def t(x) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))


def encode_ref(G_axes: np.ndarray) -> np.ndarray:
    return E.genome_to_renderer_batched(t(G_axes)).numpy()


def edge_axes_genomes() -> np.ndarray:
    """Edge cases for encode + bounds: θ at ±π / multiples of π/2 / large,
    a == b, tiny and huge scales, colours/alpha outside [0,255], off-canvas."""
    rows = []
    thetas = [0.0, math.pi, -math.pi, math.pi / 2, -math.pi / 2, math.pi / 4,
              10.0, -7.25, 100.0, 1e-8]
    scales = [(math.log(3.0), math.log(3.0)), (math.log(51.2), math.log(3.0)),
              (math.log(20.0), math.log(20.0)), (-20.0, -20.0), (-5.0, 2.0),
              (6.0, 6.0), (0.0, 0.0), (math.log(7.5), math.log(0.5))]
    rng = np.random.default_rng(123)
    for th in thetas:
        for a, b in scales:
            x, y = rng.uniform(-0.2, 1.2, 2)
            r, g, bl = rng.uniform(-40, 300, 3)
            al = rng.uniform(-10, 290)
            rows.append([x, y, a, b, th, r, g, bl, al])
    return np.asarray(rows, np.float32)[None]          # [1, 80, 9]


def raw_renderer_genomes(B, N, seed, H, W):
    """Renderer-layout genomes drawn directly (random l21, wide log range)."""
    rng = np.random.default_rng(seed)
    G = np.empty((B, N, 9), np.float32)
    G[..., 0:2] = rng.uniform(-0.1, 1.1, (B, N, 2))
    G[..., 2:4] = rng.uniform(-1.0, math.log(0.15 * max(H, W)), (B, N, 2))
    G[..., 4] = rng.uniform(-8.0, 8.0, (B, N))
    G[..., 5:8] = rng.uniform(0, 255, (B, N, 3))
    G[..., 8] = rng.uniform(120, 255, (B, N))
    return G


def main() -> None:
    meta = {"torch": torch.__version__, "triton": triton.__version__,
            "numpy": np.__version__, "python": sys.version.split()[0],
            "reference": REF, "interpreter": "TRITON_INTERPRET=1"}

    # ---- encode ------------------------------------------------------------
    enc_in = edge_axes_genomes()
    syn = synthetic_population(2, 64, 128, 128, seed=7)
    np.savez_compressed(os.path.join(HERE, "encode.npz"),
                        edge_in=enc_in, edge_out=encode_ref(enc_in),
                        syn_in=syn, syn_out=encode_ref(syn))

    # ---- preprocess ---------------------------------------------------------
    pre = {}
    cases = [("edge", encode_ref(enc_in)[0], 64, 48, 3.0),
             ("syn512", encode_ref(synthetic_population(1, 256, 512, 512, seed=11))[0], 512, 512, 3.0),
             ("raw", raw_renderer_genomes(1, 200, 5, 100, 70)[0], 100, 70, 3.0),
             ("k2", encode_ref(synthetic_population(1, 64, 90, 130, seed=3))[0], 90, 130, 2.0),
             ("w1", raw_renderer_genomes(1, 16, 9, 5, 1)[0], 5, 1, 3.0)]
    for name, g9, H, W, k in cases:
        p = R._preprocess_genome(t(g9), H, W, k, CPU)
        pre[f"{name}__in"] = g9
        pre[f"{name}__HWk"] = np.array([H, W, k], np.float64)
        for key, v in p.items():
            pre[f"{name}__{key}"] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "preprocess.npz"), **pre)

    # ---- renders -------------------------------------------------------------
    def save_render(name, G, H, W, k=3.0, bg=(1.0, 1.0, 1.0), tiles=(32,)):
        imgs = {}
        for tl in tiles:
            imgs[f"img_t{tl}"] = ref_render_cpu(t(G), H, W, k_sigma=k, background=bg,
                                                tile=tl).numpy()
        np.savez_compressed(os.path.join(HERE, f"render_{name}.npz"), genomes=G,
                            HWk=np.array([H, W, k], np.float64),
                            bg=np.asarray(bg, np.float32), **imgs)
        print("render", name, G.shape, H, W, sorted(imgs))

    save_render("64x64_n16_b2", encode_ref(synthetic_population(2, 16, 64, 64, seed=1)),
                64, 64, tiles=(16, 32, 64))
    save_render("100x70_n40_b3", encode_ref(synthetic_population(3, 40, 100, 70, seed=2)), 100, 70)
    save_render("33x47_n24_b2", encode_ref(synthetic_population(2, 24, 33, 47, seed=3)), 33, 47,
                tiles=(16, 32))
    prewarm = np.array([[[0.5, 0.5, math.log(2.0), math.log(2.0), 0.0,
                          128.0, 128.0, 128.0, 255.0]]], np.float32)   # utils.py:77-78
    save_render("prewarm_8x8", prewarm, 8, 8)
    save_render("2d_input", encode_ref(synthetic_population(1, 12, 40, 40, seed=4))[0], 40, 40)
    g12 = np.concatenate([encode_ref(synthetic_population(2, 20, 48, 48, seed=5)),
                          np.full((2, 20, 3), 77.0, np.float32)], axis=-1)
    save_render("c12", g12, 48, 48)
    save_render("black_bg", encode_ref(synthetic_population(1, 20, 48, 56, seed=6)), 48, 56,
                bg=(0.0, 0.0, 0.0))
    save_render("grey_bg_k2", encode_ref(synthetic_population(1, 20, 48, 56, seed=16)), 48, 56,
                k=2.0, bg=(0.25, 0.5, 0.75))
    save_render("edge", encode_ref(enc_in), 64, 48)
    save_render("raw", raw_renderer_genomes(2, 60, 8, 72, 96), 72, 96, tiles=(16, 64))
    save_render("128x128_n32_b8", encode_ref(synthetic_population(8, 32, 128, 128, seed=42)), 128, 128)
    save_render("tiny_5x1", raw_renderer_genomes(1, 16, 9, 5, 1), 5, 1)

    # ---- fitness -----------------------------------------------------------------
    F.render_splats_rgb_triton = ref_render_cpu     # fitness.py:4 imports the name
    fit = {}
    rng = np.random.default_rng(99)
    for name, (B, N, H, W) in {"f64": (5, 16, 64, 64), "f128": (8, 32, 128, 128),
                               "f40x56": (3, 20, 40, 56)}.items():
        pop = synthetic_population(B, N, H, W, seed=B * 1000 + N)
        target = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
        mask = M.compute_importance_mask(t(target), H, W, edge_scales=(1, 2, 4),
                                         w_edge=0.7, w_var=0.3, gamma=0.7, floor=0.15,
                                         smooth=3, strength=0.7).numpy()   # algorithm.py:42-49
        plist = [t(p) for p in pop]
        fit[f"{name}__pop"] = pop
        fit[f"{name}__target"] = target
        fit[f"{name}__mask"] = mask
        fit[f"{name}__HW"] = np.array([H, W], np.int32)
        fit[f"{name}__none"] = F.fitness_many(plist, t(target), H, W, 3.0, CPU).numpy()
        fit[f"{name}__weighted"] = F.fitness_many(plist, t(target), H, W, 3.0, CPU,
                                                  weight_mask=t(mask)).numpy()
        fit[f"{name}__boost"] = F.fitness_many(plist, t(target), H, W, 3.0, CPU,
                                               weight_mask=t(mask), boost_only=True).numpy()
        fit[f"{name}__pop_chunk2"] = np.asarray(F.fitness_population(
            plist, t(target), H, W, 3.0, CPU, tile=32, chunk=2, weight_mask=t(mask)),
            np.float64)
        print("fitness", name, fit[f"{name}__weighted"])
    np.savez_compressed(os.path.join(HERE, "fitness.npz"), **fit)

    # ---- importance mask (next-tier input) -----------------------------------------
    tgt = np.random.default_rng(5).uniform(0, 1, (96, 80, 3)).astype(np.float32)
    mk = {"target": tgt}
    for strength in (1.0, 0.7):
        mk[f"mask_s{strength}"] = M.compute_importance_mask(
            t(tgt), 96, 80, edge_scales=(1, 2, 4), w_edge=0.7, w_var=0.3, gamma=0.7,
            floor=0.15, smooth=3, strength=strength).numpy()
    # resize inside the mask (target 100x70 -> mask 64x48) and the GA's target prep
    # (algorithm.py:33-39: /255 when max > 1.5, bilinear align_corners=False)
    tgt2 = np.random.default_rng(8).uniform(0, 255, (100, 70, 3)).astype(np.float32)
    mk["target_u8"] = tgt2
    mk["mask_resized_64x48"] = M.compute_importance_mask(
        t(tgt2), 64, 48, edge_scales=(1, 2, 4), w_edge=0.7, w_var=0.3, gamma=0.7,
        floor=0.15, smooth=3, strength=0.7).numpy()
    tt = t(tgt2) / 255.0
    mk["target_prep_64x48"] = torch.nn.functional.interpolate(
        tt.permute(2, 0, 1).unsqueeze(0), size=(64, 48), mode="bilinear",
        align_corners=False)[0].permute(1, 2, 0).contiguous().numpy()
    mk["target_prep_150x90"] = torch.nn.functional.interpolate(
        tt.permute(2, 0, 1).unsqueeze(0), size=(150, 90), mode="bilinear",
        align_corners=False)[0].permute(1, 2, 0).contiguous().numpy()
    np.savez_compressed(os.path.join(HERE, "mask.npz"), **mk)

    with open(os.path.join(HERE, "meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    print("done")


if __name__ == "__main__":
    main()
