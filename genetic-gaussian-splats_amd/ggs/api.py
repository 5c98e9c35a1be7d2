"""Host side of the hot path: numpy in, numpy out, libggs.so (HIP, gfx950) underneath.

Mirrors the reference operator interface (modules/render.py, modules/fitness.py,
modules/encode.py) with plain Python + numpy; torch tensors are accepted by duck
typing (``.detach().cpu().numpy()``) so the reference's own callers work
unchanged.  Every compute call goes through ctypes into libggs.so.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import GGSInputError, check, lib

_f32p = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)


def as_f32(x) -> np.ndarray:
    """float32, C-contiguous host array from numpy / lists / torch tensors."""
    if hasattr(x, "detach") and hasattr(x, "cpu"):          # torch.Tensor (duck-typed)
        x = x.detach().cpu().numpy()
    return np.ascontiguousarray(x, dtype=np.float32)


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_f32p)


def _genomes3d(genomes, what: str) -> np.ndarray:
    g = as_f32(genomes)
    if g.ndim not in (2, 3):                                  # render.py:219
        raise GGSInputError(f"genomes must be [B,N,9] or [N,9], got {tuple(g.shape)}")
    if g.ndim == 2:                                           # render.py:220-221
        g = g[None]
    if g.shape[2] < 9:                                        # render.py:223
        raise GGSInputError(f"expected at least 9 genome cols, got {g.shape[2]} ({what})")
    return g


def device_index(device=None) -> int:
    """The HIP device a reference-style ``device`` argument names (render.py:215-217
    resolves ``device or 'cuda'`` the same way): an explicit index ('cuda:k',
    torch.device('cuda', k), k) wins; without one, LOCAL_RANK under a launcher
    (one process per GPU), else device 0.  Never "every GPU"."""
    idx = None
    if isinstance(device, int):
        idx = device
    elif isinstance(device, str):
        parts = device.split(":")
        if len(parts) == 2 and parts[1].strip().isdigit():
            idx = int(parts[1])
    elif device is not None:                                   # torch.device (duck-typed)
        idx = getattr(device, "index", None)
    if idx is None:
        idx = int(os.environ.get("LOCAL_RANK", "0") or 0)
    return int(idx)


@contextlib.contextmanager
def _on_devices(device, n_devices: int):
    """Point the host API at the devices of one call and yield the n_devices
    argument for the C layer; the selection and the call happen under one lock
    (another thread, or a direct ``ggs.select_devices``, cannot change the
    library's device list in between).  n_devices == 1 (default): the single
    device ``device`` names; n_devices > 1: fan the batch out over the first
    n_devices GPUs (opt-in; one RCCL gather returns the scalars); n_devices <= 0:
    all GPUs.

    The lock is process-wide and held for the whole C call, so the host API
    (render / fitness / encode / preprocess) is serialised across Python threads:
    concurrent host-API calls run one after another (the library's per-device
    pipeline is one stream anyway).  Threads that want concurrent GPU work use the
    device-pointer API (``fitness_device`` / ``TargetPlan`` on their own HIP
    streams), which takes no such lock."""
    n = _lib.ensure_init()
    if n_devices == 1:
        ids = (device_index(device),)
        if not 0 <= ids[0] < n:
            raise _lib.GGSDeviceError(f"device {device!r} -> HIP device {ids[0]}, but {n} visible")
    else:
        ids = tuple(range(n if n_devices <= 0 else min(int(n_devices), n)))
    with _lib.device_lock:
        if _lib.selected[0] != ids:
            _lib.select_devices(list(ids))
        yield len(ids)


def render(genomes, H: int, W: int, *, k_sigma: float = 3.0,
           background=(1.0, 1.0, 1.0), device=None, n_devices: int = 1,
           fp16_canvas: bool = False) -> np.ndarray:
    """render.py:203-252 → float32 [B,H,W,3] in [0,1] (renderer-layout genomes).

    ``fp16_canvas`` (render.py:213 ``use_fp16_canvas``): the reference's canvas is
    then float16 — the background is stored in half precision, the Triton kernel
    blends in fp32 registers and stores each pixel once as float16 (round to
    nearest even), then clamps and converts back (render.py:234-237, :252).
    Here: background rounded to half, fp32 render, result rounded to half."""
    g = _genomes3d(genomes, "render")
    B, N, Cc = g.shape
    H, W = int(H), int(W)
    out = np.empty((B, H, W, 3), np.float32)
    bg = np.ascontiguousarray(np.broadcast_to(np.asarray(background, np.float32), (3,)))
    if fp16_canvas:
        bg = bg.astype(np.float16).astype(np.float32)
    with _on_devices(device, n_devices) as nd:
        check(lib.ggs_render(_fp(g), B, N, Cc, H, W, float(k_sigma), _fp(bg), _fp(out), nd),
              "ggs_render")
    if fp16_canvas:
        out = out.astype(np.float16).astype(np.float32)
    return out


def fitness(genomes_axes, target, H: int, W: int, k_sigma: float = 3.0,
            weight_mask=None, boost_only: bool = False, boost_beta: float = 1.0,
            device=None, n_devices: int = 1) -> np.ndarray:
    """fitness.py:7-31 on a stacked [B,N,C] axes-angle batch → float32 [B]
    (on the GPU ``device`` names; ``n_devices`` > 1 opts into the multi-GPU
    fan-out, see ``_on_devices``)."""
    g = _genomes3d(genomes_axes, "fitness")
    B, N, Cc = g.shape
    H, W = int(H), int(W)
    tgt = as_f32(target)
    if tgt.shape != (H, W, 3):
        raise GGSInputError(f"target must be [H,W,3] = {(H, W, 3)}, got {tuple(tgt.shape)}")
    if weight_mask is None:
        mode, mask_p = _lib.GGS_FIT_NONE, None
    else:
        mask = as_f32(weight_mask)
        if mask.shape != (H, W):
            raise GGSInputError(f"weight_mask must be [H,W] = {(H, W)}, got {tuple(mask.shape)}")
        mode = _lib.GGS_FIT_BOOST if boost_only else _lib.GGS_FIT_WEIGHTED
        mask_p = _fp(mask)
    out = np.empty((B,), np.float32)
    with _on_devices(device, n_devices) as nd:
        check(lib.ggs_fitness(_fp(g), B, N, Cc, _fp(tgt), mask_p, mode, float(boost_beta), H, W,
                              float(k_sigma), _fp(out), nd), "ggs_fitness")
    return out


def encode(G_axes) -> np.ndarray:
    """encode.py:62-79 genome_to_renderer_batched (any leading shape, C ≥ 9) → [..., 9]."""
    g = as_f32(G_axes)
    if g.ndim == 1:
        g = g[None]
    if g.shape[-1] < 9:
        raise GGSInputError(f"expected at least 9 genome cols, got {g.shape[-1]}")
    lead = g.shape[:-1]
    flat = np.ascontiguousarray(g.reshape(-1, g.shape[-1]))
    out = np.empty((flat.shape[0], 9), np.float32)
    with _on_devices(None, 1):
        check(lib.ggs_encode(_fp(flat), flat.shape[0], flat.shape[1], _fp(out)), "ggs_encode")
    return out.reshape(*lead, 9)


def preprocess(genome, H: int, W: int, k_sigma: float = 3.0) -> Dict[str, np.ndarray]:
    """render.py:8-47 _preprocess_genome → dict of the 13 per-splat arrays."""
    g = as_f32(genome)
    if g.ndim == 1:
        g = g[None]
    g = np.ascontiguousarray(g.reshape(-1, g.shape[-1]))
    S = g.shape[0]
    f9 = np.empty((9, S), np.float32)
    i4 = np.empty((4, S), np.int32)
    with _on_devices(None, 1):
        check(lib.ggs_preprocess(_fp(g), S, g.shape[1], int(H), int(W), float(k_sigma), _fp(f9),
                                 i4.ctypes.data_as(_i32p)), "ggs_preprocess")
    keys = ("cx", "cy", "sxx", "sxy", "syy", "rc", "gc", "bc", "a")
    out = {k: f9[i] for i, k in enumerate(keys)}
    out.update({k: i4[i] for i, k in enumerate(("x0", "x1", "y0", "y1"))})
    return out


def fitness_population(population: Sequence, target, H: int, W: int, k_sigma: float = 3.0,
                       chunk: Optional[int] = None, weight_mask=None,
                       boost_only: bool = False, device=None, n_devices: int = 1) -> List[float]:
    """fitness.py:34-47 → List[float]; chunking only bounds the batch size."""
    if len(population) == 0:
        return []
    G = np.stack([as_f32(p) for p in population], 0)
    if chunk is None or chunk >= len(population):
        return fitness(G, target, H, W, k_sigma, weight_mask, boost_only,
                       device=device, n_devices=n_devices).tolist()
    out: List[float] = []
    for i in range(0, len(population), int(chunk)):
        out.extend(fitness(G[i:i + chunk], target, H, W, k_sigma, weight_mask, boost_only,
                           device=device, n_devices=n_devices).tolist())
    return out


# ---- device-pointer entry points (inputs resident in HBM) ----------------------
def fitness_device(device: int, stream: int, d_genomes: int, B: int, N: int, Cc: int,
                   d_target: int, d_mask: int, mode: int, boost_beta: float, H: int, W: int,
                   k_sigma: float, d_out: int) -> None:
    """Enqueue the fused fitness pipeline on `stream` over device pointers."""
    check(lib.ggs_fitness_device(device, C.c_void_p(stream), C.c_void_p(d_genomes), B, N, Cc,
                                 C.c_void_p(d_target), C.c_void_p(d_mask or None), mode,
                                 float(boost_beta), H, W, float(k_sigma), C.c_void_p(d_out)),
          "ggs_fitness_device")


class TargetPlan:
    """A target/mask prepared once for ``ggs_fitness_device_planned`` (the GA's
    fixed target over a run).  Pointers are device pointers on ``device``; the
    plan is built on ``stream``."""

    def __init__(self, device: int, stream: int, d_target: int, d_mask: int, mode: int,
                 boost_beta: float, H: int, W: int):
        h = C.c_void_p()
        check(lib.ggs_plan_create(device, C.c_void_p(stream), C.c_void_p(d_target),
                                  C.c_void_p(d_mask or None), mode, float(boost_beta), H, W,
                                  C.byref(h)), "ggs_plan_create")
        self.h, self.H, self.W = h, H, W

    def fitness_device(self, stream: int, d_genomes: int, B: int, N: int, Cc: int,
                       k_sigma: float, d_out: int) -> None:
        check(lib.ggs_fitness_device_planned(self.h, C.c_void_p(stream), C.c_void_p(d_genomes), B,
                                             N, Cc, float(k_sigma), C.c_void_p(d_out)),
              "ggs_fitness_device_planned")

    def close(self) -> None:
        if getattr(self, "h", None):
            lib.ggs_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 — interpreter shutdown
            pass


def render_device(device: int, stream: int, d_genomes: int, B: int, N: int, Cc: int, H: int,
                  W: int, k_sigma: float, d_out: int, background=(1.0, 1.0, 1.0)) -> None:
    bg = np.ascontiguousarray(np.broadcast_to(np.asarray(background, np.float32), (3,)))
    check(lib.ggs_render_device(device, C.c_void_p(stream), C.c_void_p(d_genomes), B, N, Cc, H,
                                W, float(k_sigma), _fp(bg), C.c_void_p(d_out)),
          "ggs_render_device")


def profile_enable(on: bool = True) -> None:
    check(lib.ggs_profile_enable(1 if on else 0), "ggs_profile_enable")


def profile_read(kernel: str):
    ms, n = C.c_double(0.0), C.c_int64(0)
    check(lib.ggs_profile_read(kernel.encode(), C.byref(ms), C.byref(n)), "ggs_profile_read")
    return ms.value, n.value


def profile_reset() -> None:
    lib.ggs_profile_reset()

