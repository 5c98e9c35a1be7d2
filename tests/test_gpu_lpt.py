"""Single-round packing of the device GA's raster launch (ggs_lpt_pack / the
breed's per-strip costs, csrc/ggs_kernels.hip lpt_kernel).

The raster's bits never depend on which block runs a strip, so the packing has to
be (1) a permutation of the launch's strips — a strip run twice or never would
corrupt the folded finalize's per-candidate count — and (2) balanced: blocks r,
r + S, r + 2S share SIMD r, and the launch ends with the largest per-SIMD sum.
The GA with and without it is compared bit for bit in
test_gpu_ga.py::test_device_ga_fused_breed_equals_unfused (the shipped shape,
where it applies)."""
from __future__ import annotations

import numpy as np
import pytest

import ggs

pytestmark = pytest.mark.gpu


def _host_rounds(c, S):
    """The packing rule restated on the host with an exact sort (reference for the
    balance bound; the device sorts into 2,048 buckets)."""
    n = c.size
    order = np.argsort(-c, kind="stable")
    load = c[order[:S]] + c[order[2 * S - 1 - np.arange(S)]]
    asc = np.argsort(load, kind="stable")
    m = n - 2 * S
    load = load.astype(np.int64)
    load[asc[:m]] += c[order[2 * S:2 * S + m]]
    return load.max()


def _simd_loads(c, mp, S):
    n = c.size
    L = np.zeros(S, np.int64)
    for k in range(3):
        r = np.arange(S)
        i = r + k * S
        ok = i < n
        L[r[ok]] += c[mp[i[ok]]]
    return L


@pytest.mark.parametrize("n,S", [(3072, 1024), (2500, 1024), (2049, 1024), (3000, 1000), (700, 256)])
@pytest.mark.parametrize("dist", ["uniform", "heavy", "constant"])
def test_lpt_pack_is_a_balanced_permutation(n, S, dist):
    rng = np.random.default_rng(n + S)
    if dist == "uniform":
        c = rng.integers(300, 6000, n)
    elif dist == "heavy":
        c = (300 + 40 * rng.pareto(1.5, n)).astype(np.int64)
    else:
        c = np.full(n, 777)
    c = c.astype(np.int32)
    mp = ggs.lpt_pack(c, S)
    np.testing.assert_array_equal(np.sort(mp), np.arange(n))
    L = _simd_loads(c.astype(np.int64), mp, S)
    host = _host_rounds(c.astype(np.int64), S)
    # the 2,048-bucket sort may swap strips within 1/2,048 of the largest cost
    assert L.max() <= host + 3 * (int(c.max()) // 2047 + 1), (L.max(), host)
    # and within 15 % of a lower bound on any packing (the greedy's worst case here
    # is uniform costs, 1.12): the mean, the largest strip with the smallest one or
    # two others (every SIMD runs 2-3 strips), the three smallest (some SIMD runs 3)
    cs = np.sort(c.astype(np.int64))
    lb = max(cs.sum() / S, cs[-1] + cs[0] + (cs[1] if n == 3 * S else 0), cs[:3].sum())
    assert L.max() <= 1.15 * lb, (L.max(), lb)


def test_lpt_pack_cost_add_and_rejects_other_shapes():
    c = np.random.default_rng(1).integers(0, 1000, 3000).astype(np.int32)
    mp = ggs.lpt_pack(c, 1024, cost_add=500)
    np.testing.assert_array_equal(np.sort(mp), np.arange(3000))
    for n, S in ((2048, 1024), (3073, 1024), (5000, 2000)):
        with pytest.raises(ValueError):
            ggs.lpt_pack(np.ones(n, np.int32), S)
    assert ggs.lpt_pack(np.zeros(0, np.int32), 1024).size == 0
