"""Host-side semantics the drop-ins owe the reference's callers (CPU, no GPU):

* seeding: run_ggs.py:25-28 / run_sags.py:26-27 call ``random.seed(SEED)`` and
  expect a repeatable run — with ``seed=None`` every draw source derives its seed
  from Python's ``random`` (ggs.ga.resolve_seed);
* ``device`` (render.py:215-217): 'cuda:k' names device k; without an index the
  launcher's LOCAL_RANK, else 0 — never "every GPU";
* the torch-free RCCL id exchange (ggs.parallel.file_rendezvous) across real
  processes, as the ranks of one node use it.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import random

import numpy as np
import pytest

from ggs import annealing as A
from ggs import api, ga
from ggs.parallel import file_rendezvous

SIG_MAX = {"xy": 0.08, "alog": 0.3, "blog": 0.3, "theta": 0.6, "rgb": 40.0, "alpha": 30.0}
SIG_MIN = {"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.1, "rgb": 5.0, "alpha": 5.0}


def _energy(G):
    """A cheap deterministic stand-in evaluator (the GA's plumbing, not the raster)."""
    G = np.asarray(G, np.float64)
    return (np.sin(G[..., 0] * 3.0 + G[..., 4]).sum(-1) + 0.01 * G[..., 5:9].mean((-1, -2))).astype(np.float32)


def _ga_run():
    tgt = np.random.default_rng(0).uniform(0, 1, (24, 20, 3)).astype(np.float32)
    return ga.genetic_approx(tgt, 24, 20, "cuda", 8, 12, 3, 2, 2, 0.7, 0.3, SIG_MAX, SIG_MIN,
                             "cosine", 3.0, 0.1, 3.0, 0.7, False, evaluate=_energy,
                             progress=False, return_state=True, backend="host")


def test_random_seed_makes_the_host_ga_repeatable():
    random.seed(42)
    a = _ga_run()
    random.seed(42)
    b = _ga_run()
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[2]["population"], b[2]["population"])
    assert a[1] == b[1]
    random.seed(43)
    c = _ga_run()
    assert not np.array_equal(a[2]["population"], c[2]["population"])


def test_random_seed_makes_the_host_sa_repeatable():
    tgt = np.random.default_rng(1).uniform(0, 1, (16, 16, 3)).astype(np.float32)

    def run():
        return A.simulated_annealing(tgt, 16, 16, "cuda", n_splats=10, mutpb=0.2,
                                     mut_sigma_max=SIG_MAX, mut_sigma_min=SIG_MIN,
                                     sigma_schedule="linear", min_scale_splats=3.0,
                                     max_scale_splats=0.1, k_sigma=3.0, mask_strength=0.7,
                                     boost_only=False, iterations=6, temp0=1e-2,
                                     temp_schedule="exp", tries_per_iter=3,
                                     evaluate=_energy, progress=False, return_state=True,
                                     backend="host")
    random.seed(7)
    a = run()
    random.seed(7)
    b = run()
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[2]["current"], b[2]["current"])


def test_resolve_seed_follows_random_state():
    random.seed(5)
    s1 = ga.resolve_seed(None)
    random.seed(5)
    assert ga.resolve_seed(None) == s1
    assert ga.resolve_seed(123) == 123


def test_module_draw_sources_made_at_import_follow_a_later_random_seed():
    d1, d2 = ga.NumpyDraws(), ga.NumpyDraws()          # made before the seed, like module globals
    random.seed(11)
    x = d1.uniform(5)
    random.seed(11)
    np.testing.assert_array_equal(x, d2.uniform(5))


def test_population_module_rng_follows_random_seed():
    import importlib
    import modules.population as P
    importlib.reload(P)
    random.seed(3)
    a = P.new_population(2, 4, 16, 16, 3.0, 0.1)
    importlib.reload(P)
    random.seed(3)
    b = P.new_population(2, 4, 16, 16, 3.0, 0.1)
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("device, env, want", [
    ("cuda:3", None, 3), ("cuda:0", "5", 0), (2, "5", 2), ("cuda", None, 0), (None, None, 0),
    ("cuda", "6", 6), (None, "1", 1),
])
def test_device_argument_names_one_gpu(monkeypatch, device, env, want):
    if env is None:
        monkeypatch.delenv("LOCAL_RANK", raising=False)
    else:
        monkeypatch.setenv("LOCAL_RANK", env)
    assert api.device_index(device) == want


def test_device_argument_accepts_torch_devices():
    torch = pytest.importorskip("torch")
    assert api.device_index(torch.device("cuda", 4)) == 4
    assert api.device_index(torch.device("cuda:1")) == 1


def _rdzv_rank(rank, world, key, d, q):
    idb = file_rendezvous(rank, world, lambda: bytes(range(128)) if rank == 0 else b"", key=key,
                          directory=d, timeout_s=30)
    q.put((rank, idb))


def test_file_rendezvous_carries_rank0s_id_to_every_rank(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 3
    procs = [ctx.Process(target=_rdzv_rank, args=(r, world, f"t{os.getpid()}", str(tmp_path), q))
             for r in (2, 1, 0)]                        # the readers start first
    for p in procs:
        p.start()
    got = dict(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert set(got) == {0, 1, 2} and all(v == bytes(range(128)) for v in got.values())


def test_file_rendezvous_times_out_without_rank0(tmp_path):
    with pytest.raises(TimeoutError):
        file_rendezvous(1, 2, lambda: b"", key="nobody", directory=str(tmp_path), timeout_s=0.2)


def _philox_u53(seed: int, it: int, k: int) -> float:
    """Philox4x32-10 (Salmon et al., SC'11) on counter (it, k, 0, 8), key = seed,
    restated in Python integers: the acceptance uniform the device SA loop draws."""
    M = 0xFFFFFFFF
    c = [it & M, k & M, 0, 8]
    k0, k1 = seed & M, (seed >> 32) & M
    for _ in range(10):
        p0, p1 = 0xD2511F53 * c[0], 0xCD9E8D57 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & M, p1 & M, ((p0 >> 32) ^ c[3] ^ k1) & M, p0 & M]
        k0, k1 = (k0 + 0x9E3779B9) & M, (k1 + 0xBB67AE85) & M
    return ((c[0] >> 5) * 67108864.0 + (c[1] >> 6)) / 9007199254740992.0


def test_sa_accept_uniform_is_philox():
    """ggs_sa_accept_uniform (host code in libggs, the same function the device
    loop's accept kernel calls) against an independent restatement."""
    from ggs.ga_device import PhiloxAcceptDraws
    for seed in (0, 42, 2**63 + 12345):
        d = PhiloxAcceptDraws(seed)
        us = [d.accept_at(it, k) for it in (0, 1, 7, 1000) for k in range(5)]
        assert us == [_philox_u53(seed, it, k) for it in (0, 1, 7, 1000) for k in range(5)]
        assert all(0.0 <= u < 1.0 for u in us) and len(set(us)) == len(us)
    with pytest.raises(Exception):
        PhiloxAcceptDraws(0).accept_at(-1, 0)


def test_host_api_reselects_after_a_direct_select_devices(monkeypatch):
    """``ggs.select_devices`` and the host API share one view of the library's
    device list: after a direct selection the next call re-selects its own
    device, and the selection and the call happen under one lock."""
    from ggs import _lib, api
    calls = []

    class FakeLib:
        def ggs_select_devices(self, arr, n):
            calls.append([arr[i] for i in range(n)])
            assert _lib.device_lock._is_owned()
            return n

    monkeypatch.setattr(_lib, "lib", FakeLib())
    monkeypatch.setattr(_lib, "ensure_init", lambda: 2)
    monkeypatch.setattr(_lib, "selected", [None])
    with api._on_devices("cuda:0", 1) as nd:
        assert nd == 1 and _lib.device_lock._is_owned()
    with api._on_devices(0, 1):
        pass                                   # cached: no second selection
    _lib.select_devices([1])                   # a caller points the library elsewhere
    with api._on_devices(0, 1):
        pass
    with api._on_devices(None, 0) as nd:       # all devices
        assert nd == 2
    assert calls == [[0], [1], [0], [0, 1]]
