"""Register budget of the shipped kernels, read from libggs.so's own code objects
(tools/kernel_resources.py: the AMDHSA metadata notes; CPU only, no rebuild).

The raster is sized for 3 waves per SIMD (<= 168 VGPRs, csrc/ggs_kernels.hip
OCC): a 169th VGPR drops it to 2 waves, and a spill puts scratch traffic into
the epilogue (round 4: the folded-finalize instances spilled 2 VGPRs, 12 B/lane,
without any test noticing)."""
from __future__ import annotations

import importlib.util
import os

import pytest

from conftest import REPO


def _tool():
    spec = importlib.util.spec_from_file_location(
        "kernel_resources", os.path.join(REPO, "tools", "kernel_resources.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.fixture(scope="module")
def res():
    import ggs
    return _tool().kernel_resources(ggs.LIB_PATH)


def test_every_raster_instance_fits_three_waves_without_scratch(res):
    raster = {n: r for n, r in res.items() if "raster_kernel" in n}
    # image / fitness / fitness + folded finalize, each with and without the
    # saturation cut-off
    assert len(raster) == 6, sorted(raster)
    for n, r in raster.items():
        assert r["vgpr_count"] <= 168, (n, r)
        assert r["waves_per_simd"] == 3, (n, r)
        assert r["private_segment_fixed_size"] == 0, (n, r)
        assert r["vgpr_spill_count"] == 0 and r["sgpr_spill_count"] == 0, (n, r)
        assert r["wavefront_size"] == 64, (n, r)


def test_no_kernel_uses_scratch(res):
    assert len(res) >= 20
    bad = {n: r["private_segment_fixed_size"] for n, r in res.items() if r["private_segment_fixed_size"]}
    assert not bad, bad
    assert all(r["vgpr_spill_count"] == 0 for r in res.values())
