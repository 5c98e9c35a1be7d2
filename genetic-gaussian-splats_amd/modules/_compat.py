"""Shared plumbing of the drop-in modules: locate ``ggs`` and hand results
back in the caller's array type (numpy in → numpy out; torch in → torch out on
the caller's device, without importing torch for numpy callers)."""
from __future__ import annotations

import os
import sys

try:
    import ggs  # noqa: F401
except ImportError:  # modules/ copied next to the reference: find the sibling package
    sys.path.insert(0, os.environ.get(
        "GGS_HOME", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    import ggs  # noqa: F401


def is_torch(x) -> bool:
    return type(x).__module__.split(".")[0] == "torch"


def like(out, ref):
    """Return numpy `out` as the same kind of array as `ref` (torch → torch)."""
    if is_torch(ref):
        torch = sys.modules["torch"]
        return torch.from_numpy(out).to(ref.device)
    return out


def first(seq):
    return seq[0] if len(seq) else None


def check_device(device) -> None:
    """render.py:215-217: the reference asserts a CUDA (here: HIP) device."""
    if device is None:
        return
    kind = getattr(device, "type", None) or str(device).split(":")[0]
    if kind != "cuda":
        raise ggs.GGSInputError("This renderer requires a CUDA device.")


def hip_device_of(*xs):
    """Device index when every x is a torch tensor on the same HIP ("cuda")
    device, else None: such inputs take the device-pointer path (no PCIe copy)."""
    dev = None
    for x in xs:
        if x is None:
            continue
        if not is_torch(x) or x.device.type != "cuda":
            return None
        idx = x.device.index if x.device.index is not None else \
            sys.modules["torch"].cuda.current_device()
        if dev is not None and idx != dev:
            return None
        dev = idx
    return dev


def f32_contig(x):
    """torch tensor -> contiguous float32 (same device)."""
    torch = sys.modules["torch"]
    return x.detach().to(torch.float32).contiguous()


def stream_of(dev: int) -> int:
    return sys.modules["torch"].cuda.current_stream(dev).cuda_stream
