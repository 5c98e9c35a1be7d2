"""Drop-in for the reference's modules/annealing.py (annealing.py:19-190).

``simulated_annealing`` keeps the reference signature and runs ggs/annealing.py:
the tries of an iteration are mutated in one batch and evaluated in ONE libggs
launch, accepted in order exactly as the sequential loop (proven against the
reference's recorded draws in tests/test_sa.py).  Extra keyword hooks pass
through (``seed``, ``speculate``, ...).  Returns (best individual, best energy);
the individual is a torch CPU tensor when the target was a torch tensor
(annealing.py:190 returns ``best.cpu()``).
"""
from __future__ import annotations

from modules._compat import ggs, is_torch
from ggs import annealing as _sa

_temp_schedule = _sa.temp_schedule                         # annealing.py:29-44


def simulated_annealing(target_img_uint8, H: int, W: int, device, n_splats: int, mutpb: float,
                        mut_sigma_max: dict, mut_sigma_min: dict, sigma_schedule: str,
                        min_scale_splats: float, max_scale_splats: float, k_sigma: float,
                        mask_strength: float, boost_only: bool, iterations: int, temp0: float,
                        temp_schedule: str, tries_per_iter: int = 1, save_video: bool = False,
                        frame_every: int = 10_000, video_dir: str = "", prefix: str = "sa",
                        loss_png_path: str = "", loss_csv_path: str = "",
                        loss_log_y: bool = False, **hooks):
    best, best_fit = _sa.simulated_annealing(
        ggs.as_f32(target_img_uint8), H, W, device, n_splats, mutpb, mut_sigma_max,
        mut_sigma_min, sigma_schedule, min_scale_splats, max_scale_splats, k_sigma,
        mask_strength, boost_only, iterations, temp0, temp_schedule, tries_per_iter, save_video,
        frame_every, video_dir, prefix, loss_png_path, loss_csv_path, loss_log_y, **hooks)[:2]
    if is_torch(target_img_uint8):
        import sys
        return sys.modules["torch"].from_numpy(best), best_fit
    return best, best_fit
