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
