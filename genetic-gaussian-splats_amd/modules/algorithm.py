"""Drop-in for the reference's modules/algorithm.py (algorithm.py:16-195).

``genetic_approx`` keeps the reference signature; the generation is built with
the batched operators of ggs/ga.py (numpy, one array op per gene group for the
whole population) and evaluated with ONE libggs fitness launch per generation.
Randomness: numpy Generator (``seed=`` keyword, default fresh entropy) — the
reference's torch/Python RNG streams cannot be reproduced without torch; the
operators are proven draw-for-draw identical to the reference's in
tests/test_ga.py.  Returns (best individual, best fitness); the individual is a
torch CPU tensor when the target was a torch tensor (as algorithm.py:195).
"""
from __future__ import annotations

from modules._compat import ggs, is_torch
from ggs import ga as _ga


def genetic_approx(target_img_uint8, H: int, W: int, device, pop_size: int, n_splats: int,
                   generations: int, tour_k: int, elite_k: int, cxpb: float, mutpb: float,
                   mut_sigma_max: dict, mut_sigma_min: dict, schedule: str,
                   min_scale_splats: float, max_scale_splats: float, k_sigma: float,
                   mask_strength: float, boost_only: bool, save_video: bool = False,
                   frame_every: int = 5000, video_dir: str = "", prefix: str = "ga",
                   loss_png_path: str = "", loss_csv_path: str = "", loss_log_y: bool = False,
                   **hooks):
    best, best_fit = _ga.genetic_approx(
        ggs.as_f32(target_img_uint8), H, W, device, pop_size, n_splats, generations, tour_k,
        elite_k, cxpb, mutpb, mut_sigma_max, mut_sigma_min, schedule, min_scale_splats,
        max_scale_splats, k_sigma, mask_strength, boost_only, save_video, frame_every,
        video_dir, prefix, loss_png_path, loss_csv_path, loss_log_y, **hooks)
    if is_torch(target_img_uint8):
        import sys
        return sys.modules["torch"].from_numpy(best), best_fit
    return best, best_fit
