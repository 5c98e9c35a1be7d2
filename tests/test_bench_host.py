"""bench.py's host-side pieces on CPU (no GPU): the workload's algorithmic byte
count, the synthetic population (population.py:20-46
distributions), and where the roofline's PMC traffic / VALU-busy come from."""
from __future__ import annotations

import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_algorithmic_bytes_per_candidate():
    assert (bench.H, bench.W, bench.N_SPLATS) == (512, 512, 256)
    assert bench.bytes_per_candidate() == 4_203_524          # 12HW + 4HW + 36N + 4


def test_synthetic_population_distributions():
    G = bench.synthetic_population(64, 256, 0)
    assert G.shape == (64, 256, 9) and G.dtype == np.float32
    assert (G[..., :2] >= 0).all() and (G[..., :2] <= 1).all()
    lo, hi = np.log(3.0), np.log(0.1 * 512)
    assert (G[..., 2:4] >= lo - 1e-6).all() and (G[..., 2:4] <= hi + 1e-6).all()
    assert (np.abs(G[..., 4]) <= np.pi + 1e-6).all()
    assert (G[..., 5:8] >= 0).all() and (G[..., 5:8] <= 255).all()
    assert (G[..., 8] >= 180).all() and (G[..., 8] <= 255).all()
    # a_log skews small (Beta mean 0.4), b_log large (0.6)
    assert G[..., 2].mean() < G[..., 3].mean()
    np.testing.assert_array_equal(G, bench.synthetic_population(64, 256, 0))


def test_pmc_figures_come_from_this_workloads_profile():
    paths = bench._bench_profiles()
    assert paths and all(os.path.basename(os.path.dirname(p)).startswith("r") for p in paths)
    assert not any("_" in os.path.basename(os.path.dirname(p)) for p in paths)   # not rNN_<config>
    traffic, src = bench.pmc_traffic()
    assert traffic > 0 and src.startswith("profiles/r") and src.endswith("summary.json")
    busy = bench.pmc_valu_busy()
    assert 0.3 < busy < 1.0
