"""The deterministic float32 functions shared (bit-for-bit) by the oracle and
the HIP prep stage: accuracy against float64 and the domain conventions."""
from __future__ import annotations

import numpy as np

from detmath import exp_f32, log_f32, sincos_f32


def _ulps(a, ref):
    sp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    return np.abs(a.astype(np.float64) - ref) / sp


def test_exp_accuracy():
    x = np.random.default_rng(0).uniform(-87, 88.7, 400_000).astype(np.float32)
    assert _ulps(exp_f32(x), np.exp(x.astype(np.float64))).max() < 1.0


def test_log_accuracy():
    x = np.exp(np.random.default_rng(1).uniform(-40, 40, 400_000)).astype(np.float32)
    assert _ulps(log_f32(x), np.log(x.astype(np.float64))).max() < 1.0


def test_sincos_accuracy():
    x = np.random.default_rng(2).uniform(-100, 100, 400_000).astype(np.float32)
    s, c = sincos_f32(x)
    x64 = x.astype(np.float64)
    assert np.abs(s - np.sin(x64)).max() < 2e-7
    assert np.abs(c - np.cos(x64)).max() < 2e-7


def test_domain_conventions():
    e = exp_f32(np.array([0, -87.5, 89.0, np.nan, -np.inf, np.inf], np.float32))
    assert e[0] == 1 and e[1] == 0 and np.isinf(e[2]) and np.isnan(e[3])
    assert e[4] == 0 and np.isinf(e[5])
    assert exp_f32(np.float32(-86.99)) > np.finfo(np.float32).tiny    # never subnormal
    lg = log_f32(np.array([1, 0, -1, np.inf, 1e-40], np.float32))
    assert lg[0] == 0 and lg[1] == -np.inf and np.isnan(lg[2]) and lg[3] == np.inf
    assert abs(lg[4] - np.log(1e-40)) < 1e-4
    s, c = sincos_f32(np.array([0, np.inf], np.float32))
    assert s[0] == 0 and c[0] == 1 and np.isnan(s[1]) and np.isnan(c[1])


def test_outputs_are_float32_and_shape_preserving():
    x = np.linspace(-3, 3, 12, dtype=np.float32).reshape(3, 4)
    for y in (exp_f32(x), log_f32(np.abs(x) + 1), *sincos_f32(x)):
        assert y.dtype == np.float32 and y.shape == (3, 4)
