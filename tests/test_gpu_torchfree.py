"""The north_star configuration on the GPU: plain Python + numpy over the C ABI,
no PyTorch in the process, /opt/rocm's HIP runtime (GGS_HIP_RUNTIME=system).
Runs __graft_entry__.smoke() (render + fitness vs the oracle) in a fresh
interpreter where ``import torch`` is blocked, and checks which runtime was
mapped.  Plus the drop-in's ``device`` and ``use_fp16_canvas`` semantics."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ORACLE, PKG, REPO

pytestmark = pytest.mark.gpu

_SCRIPT = r'''
import sys
sys.modules["torch"] = None                  # any "import torch" now raises ImportError
sys.path[:0] = [{repo!r}, {pkg!r}, {oracle!r}]
import __graft_entry__ as E
E.smoke()
import ggs.hip, ggs.parallel, modules.fitness, modules.render   # the torch-free host surface
maps = open("/proc/self/maps").read()
hip = sorted({{l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}})
print("HIP_RUNTIME", ";".join(hip))
print("TORCH_LIBS", sum("libtorch" in l for l in maps.splitlines()))
'''


def test_smoke_without_torch_on_the_system_hip_runtime():
    env = dict(os.environ, GGS_HIP_RUNTIME="system")
    r = subprocess.run([sys.executable, "-c", _SCRIPT.format(repo=REPO, pkg=PKG, oracle=ORACLE)],
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "smoke ok" in r.stdout
    hip = next(l for l in r.stdout.splitlines() if l.startswith("HIP_RUNTIME")).split(" ", 1)[1]
    assert hip.startswith("/opt/rocm") and "torch" not in hip, hip
    assert "TORCH_LIBS 0" in r.stdout


def test_device_argument_out_of_range_is_a_device_error():
    import ggs
    n = ggs.ensure_init()
    pop = np.zeros((1, 4, 9), np.float32)
    with pytest.raises(ggs.GGSDeviceError):
        ggs.render(pop, 8, 8, device=f"cuda:{n}")
    img = ggs.render(pop, 8, 8, device="cuda:0")
    assert img.shape == (1, 8, 8, 3)


def test_fp16_canvas_matches_the_reference_semantics():
    """render.py:234-237/252 with use_fp16_canvas=True: a float16 canvas holds the
    background; each pixel is blended in fp32 and stored once as float16; then
    clamp and back to float32.  The oracle's fp32 image rounded the same way
    agrees to within one half-precision ulp (the fp32 images differ by ~3e-6 and
    can straddle a rounding boundary)."""
    import ggs_oracle as O
    from modules.render import render_splats_rgb_triton
    H, W = 48, 56
    enc = O.genome_to_renderer_batched(O.synthetic_population(3, 20, H, W, seed=11))
    bg = (0.3, 0.6, 0.9)                                  # not representable in half precision
    got = render_splats_rgb_triton(enc, H, W, background=bg, use_fp16_canvas=True)
    assert got.dtype == np.float32
    np.testing.assert_array_equal(got, got.astype(np.float16).astype(np.float32))   # half values
    bg16 = tuple(float(np.float16(c)) for c in bg)
    ref = O.render(enc, H, W, background=bg16).astype(np.float16).astype(np.float32)
    ulp = np.spacing(np.maximum(np.abs(ref), 2.0 ** -14).astype(np.float16)).astype(np.float32)
    assert (np.abs(got - ref) <= ulp).all()
    assert (got == ref).mean() > 0.99
