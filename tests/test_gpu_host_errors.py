"""Error returns of the host API (the drop-in path on the caller's arrays) leave
nothing running against those arrays (include/ggs.h: pointers are used only
during the call).  The host API copies straight between the caller's pageable
arrays and the device, so a failure on a later shard (n_devices > 1) must not
return while an earlier shard's copies are still queued; every stream that was
given work is synchronised on every return.  One GPU here, so the failure is
injected after the first (only) device's work is queued
(GGS_TEST_FAIL_AFTER_ENQUEUE=1, read per call); afterwards the library works on."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import ggs
import ggs_oracle as O
from conftest import ORACLE, PKG

pytestmark = pytest.mark.gpu

H, W, B, N = 96, 80, 6, 40


def _inputs(seed=3):
    pop = O.synthetic_population(B, N, H, W, seed=seed)
    rng = np.random.default_rng(seed)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.4, 1.0, (H, W)).astype(np.float32)
    return pop, tgt, mask


def _p(a):
    return a.ctypes.data_as(ggs._lib._f32p)


def test_render_error_after_enqueue_leaves_the_output_alone(monkeypatch):
    pop, _, _ = _inputs()
    enc = np.ascontiguousarray(ggs.encode(pop))
    want = ggs.render(enc, H, W)
    out = np.full((B, H, W, 3), -7.0, np.float32)
    monkeypatch.setenv("GGS_TEST_FAIL_AFTER_ENQUEUE", "1")
    rc = ggs.lib.ggs_render(_p(enc), B, N, 9, H, W, 3.0, None, _p(out), 0)
    assert rc == ggs._lib.GGS_EHIP and "injected" in ggs._lib.last_error()
    snap = out.copy()
    time.sleep(0.05)
    np.testing.assert_array_equal(out, snap)          # nothing lands after the return
    assert (out == -7.0).all()                         # the image copies are queued last
    monkeypatch.delenv("GGS_TEST_FAIL_AFTER_ENQUEUE")
    np.testing.assert_array_equal(ggs.render(enc, H, W), want)


def test_fitness_error_after_enqueue_then_recovers(monkeypatch):
    pop, tgt, mask = _inputs(4)
    want = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)      # caches target / mask (speculative path)
    g = np.ascontiguousarray(pop, np.float32)
    out = np.full(B, -7.0, np.float32)
    monkeypatch.setenv("GGS_TEST_FAIL_AFTER_ENQUEUE", "1")
    rc = ggs.lib.ggs_fitness(_p(g), B, N, 9, _p(tgt), _p(mask), ggs.GGS_FIT_WEIGHTED, 1.0, H, W, 3.0, _p(out), 0)
    assert rc == ggs._lib.GGS_EHIP and "injected" in ggs._lib.last_error()
    assert (out == -7.0).all()
    monkeypatch.delenv("GGS_TEST_FAIL_AFTER_ENQUEUE")
    np.testing.assert_array_equal(ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask), want)


_GATHER = r'''
import sys, numpy as np
sys.path[:0] = [{pkg!r}, {oracle!r}]
import ggs, ggs_oracle as O
H, W, B, N = {H}, {W}, {B}, {N}
pop = O.synthetic_population(B, N, H, W, seed=5)
rng = np.random.default_rng(5)
tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
mask = rng.uniform(0.4, 1.0, (H, W)).astype(np.float32)
want = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
import os
os.environ["GGS_TEST_FAIL_AFTER_ENQUEUE"] = "1"
try:
    ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
    raise SystemExit("no error")
except ggs.GGSError as e:
    assert "injected" in str(e), e
del os.environ["GGS_TEST_FAIL_AFTER_ENQUEUE"]
np.testing.assert_array_equal(ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask), want)
print("ok")
'''


def test_fitness_gather_path_error_after_enqueue_then_recovers():
    """The fan-out path (GGS_FANOUT_RCCL=1: the RCCL gather at one device)."""
    script = _GATHER.format(pkg=PKG, oracle=ORACLE, H=H, W=W, B=B, N=N)
    r = subprocess.run([sys.executable, "-c", script], env=dict(os.environ, GGS_FANOUT_RCCL="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]
