"""Drop-in for the reference's modules/render.py (render.py:1-252).

``render_splats_rgb_triton`` keeps the reference signature; the work runs in
libggs.so (HIP, gfx950): prep + order-preserving per-tile cull + front-to-back
blend, one launch each.  ``tile``, ``num_warps`` and ``num_stages`` are accepted
and ignored — the reference output is tile-invariant and the
MI355X kernel picks its own tiling.  ``device`` selects the GPU as in the
reference ('cuda:k' → device k; 'cuda' / None → the launcher's LOCAL_RANK, else
0).  ``use_fp16_canvas`` (render.py:213, never set by a reference caller) keeps
the reference's float16-canvas semantics: background and the stored pixels
rounded to half precision (render.py:234-237), the blend in fp32.
"""
from __future__ import annotations

import sys

from modules._compat import check_device, f32_contig, ggs, hip_device_of, like, stream_of

_DEV = "cuda"   # imported by run_ggs.py:8 / run_sags.py:8; 'cuda' is ROCm's HIP device type
__all__ = ["render_splats_rgb_triton", "_DEV"]


def render_splats_rgb_triton(genomes, H: int, W: int, *, k_sigma: float = 3.0, device=None,
                             background=(1.0, 1.0, 1.0), tile: int = 64, num_warps: int = 8,
                             num_stages: int = 3, use_fp16_canvas: bool = False):
    """render.py:203-252 → [B,H,W,3] float32 clamped to [0,1] (numpy, or torch
    on the input's device when given a torch tensor)."""
    check_device(device or _DEV)
    dev = hip_device_of(genomes)
    if dev is not None:                   # torch tensor on the GPU: device pointers, no copies
        torch = sys.modules["torch"]
        if genomes.ndim not in (2, 3):
            raise ggs.GGSInputError("Expected genomes [N,C] or [B,N,C]")   # render.py:219
        g = f32_contig(genomes if genomes.ndim == 3 else genomes.unsqueeze(0))
        B, N, C = g.shape
        if C < 9:
            raise ggs.GGSInputError("Expected at least 9 genome cols")    # render.py:223
        out = torch.empty((B, H, W, 3), dtype=torch.float32, device=g.device)
        bg = torch.tensor(background, dtype=torch.float16 if use_fp16_canvas else torch.float32)
        ggs.render_device(dev, stream_of(dev), g.data_ptr(), B, N, C, H, W, k_sigma,
                          out.data_ptr(), background=bg.float().tolist())
        return out.half().float() if use_fp16_canvas else out
    out = ggs.render(genomes, H, W, k_sigma=k_sigma, background=background, device=device,
                     fp16_canvas=use_fp16_canvas)
    return like(out, genomes)
