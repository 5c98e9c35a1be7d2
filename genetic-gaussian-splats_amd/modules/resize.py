"""Drop-in for the reference's modules/resize.py (resize.py:1-20): the working
resolution and the genome rescale used for the final full-resolution render
(run_ggs.py:64-77, run_sags.py:73-88)."""
from __future__ import annotations

from typing import Tuple

import numpy as np

from modules._compat import ggs, is_torch, like


def choose_work_size(Ht: int, Wt: int, max_side: int = 128) -> Tuple[int, int]:
    """resize.py:6-13: longest side → max_side, the other rounded (Python round)."""
    if Ht >= Wt:
        Hf = max_side
        Wf = max(1, int(round(Wt * Hf / Ht)))
    else:
        Wf = max_side
        Hf = max(1, int(round(Ht * Wf / Wt)))
    return Hf, Wf


def scale_genome_pixels_anisotropic(ind, sH: float, sW: float):
    """resize.py:16-20: add log(sW) to a_log and log(sH) to b_log (float32 add of
    the float64 log, as torch's in-place add of a Python float)."""
    out = np.array(ggs.as_f32(ind), np.float32, copy=True)
    out[:, 2] += np.float32(float(np.log(sW)))
    out[:, 3] += np.float32(float(np.log(sH)))
    return like(out, ind) if is_torch(ind) else out

