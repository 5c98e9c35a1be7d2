"""The multi-GPU data-path collective through the C ABI, with no
PyTorch: ``ggs_comm_*`` all-gathers per-rank fitness scalars over RCCL on a HIP
stream (in-stream or overlapped on the communicator's own stream), the
single-process communicators of the host API's fan-out (``ggs_comm_init_local``),
and the host-side barrier / all-gather.  One GPU here, so world-1 communicators;
the N > 1 sharding logic and the file rendezvous are covered on CPU
(tests/test_dist_gloo.py, tests/test_host_semantics.py) and run at N = 2..8 by
bench.py.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

import ggs
import ggs_oracle as O
from conftest import ORACLE, PKG

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    from ggs import hip as h
    ggs.ensure_init()
    h.set_device(0)
    return h


@pytest.mark.parametrize("overlap", [False, True])
def test_rccl_allgather_returns_every_shard(hip, overlap, monkeypatch):
    monkeypatch.setenv("GGS_COMM_RCCL_SELF", "1")      # world 1: through RCCL, not the copy kernel
    comm = ggs.RcclGather(0, rank=0, world=1)
    st = hip.Stream()
    try:
        for count in (1, 128, 4099):
            x = (np.arange(count, dtype=np.float32) * 0.5 - 3.0)
            send = hip.DeviceArray.from_host(x)
            recv = hip.DeviceArray.from_host(np.full(count * comm.world, np.nan, np.float32))
            t = comm.allgather(st.handle, send.ptr, recv.ptr, count, overlap=overlap)
            assert (t >= 0) == overlap
            comm.wait(st.handle, t)
            np.testing.assert_array_equal(recv.to_host(st)[comm.rank * count:(comm.rank + 1) * count], x)
    finally:
        comm.close()


def test_rccl_reports_world1_and_one_tree(hip):
    """The rank count a run reports is RCCL's own (ncclCommCount /
    ncclCommUserRank / ncclCommCuDevice), and HIP + RCCL come from one directory."""
    comm = ggs.RcclGather(0, rank=0, world=1)
    try:
        assert comm.info() == (1, 0, 0)
        info = ggs.runtime_info()
        assert info["same_tree"] is True, info
        assert os.path.dirname(info["rccl"]) == os.path.dirname(info["hip"])
        assert info["rccl_version"] > 0 and info["hip_version"] > 0
        from ggs import _lib
        assert len(_lib.mapped("libamdhip64")) == 1 and len(_lib.mapped("librccl")) == 1
    finally:
        comm.close()
    lb = ggs.parallel.loopback_group(0, 2)
    with pytest.raises(ggs.GGSInputError):            # no RCCL behind a loopback rank
        lb[0].info()
    for g in lb:
        g.close()


_COMM_THEN_TORCH = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import ggs
from ggs import hip
comm = ggs.RcclGather(0, rank=0, world=1)
st = hip.Stream()
x = hip.DeviceArray.from_host(np.arange(64, dtype=np.float32))
y = hip.DeviceArray((64,))
comm.allgather(st.handle, x.ptr, y.ptr, 64)
assert (y.to_host(st) == np.arange(64)).all()
comm.close()
import torch
print("ok", torch.__version__)
"""


def test_comm_then_torch_exits_cleanly():
    """Round 5's exit abort (a communicator made, torch imported afterwards):
    status 0 and no allocator error now that RCCL is loaded RTLD_LOCAL."""
    r = subprocess.run([sys.executable, "-c", _COMM_THEN_TORCH, PKG], capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, GGS_COMM_RCCL_SELF="1"))
    assert r.returncode == 0 and "ok" in r.stdout, (r.returncode, r.stderr[-2000:])
    assert "double free" not in r.stderr and "free()" not in r.stderr


def test_host_allgather_and_barrier(hip):
    comm = ggs.RcclGather(0, rank=0, world=1)
    try:
        v = np.array([1.5, -2.0, 3.25], np.float32)
        got = comm.allgather_host(v)
        assert got.shape == (1, 3)
        np.testing.assert_array_equal(got[0], v)
        # bit patterns survive (fingerprints travel as float32 pairs)
        raw = np.array([0x7FC00001, 0xFFFFFFFF], np.uint32).view(np.float32)
        assert comm.allgather_host(raw).view(np.uint32).tolist() == [[0x7FC00001, 0xFFFFFFFF]]
        comm.barrier()
    finally:
        comm.close()


def test_sharded_fitness_through_rccl_matches_oracle(hip):
    """bench.py's step: fused fitness of this rank's candidates into a ring slot,
    overlapped gather, join — the gathered vector equals the oracle's fitness."""
    H = W = 64
    B, N = 6, 12
    pop = O.synthetic_population(B, N, H, W, seed=7)
    rng = np.random.default_rng(3)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.4, 1.0, (H, W)).astype(np.float32)
    g, t_d, m_d = (hip.DeviceArray.from_host(a) for a in (pop, tgt, mask))
    out = hip.DeviceArray((B,))
    st = hip.Stream()
    comm = ggs.RcclGather(0, rank=0, world=1)
    try:
        plan = ggs.TargetPlan(0, st.handle, t_d.ptr, m_d.ptr, ggs.GGS_FIT_WEIGHTED, 1.0, H, W)
        plan.fitness_device(st.handle, g.ptr, B, N, 9, 3.0, out.ptr)
        full = hip.DeviceArray((B * comm.world,))
        comm.wait(st.handle, comm.allgather(st.handle, out.ptr, full.ptr, B, overlap=True))
        got = full.to_host(st)[:B]
    finally:
        comm.close()
    ref = np.asarray(O.fitness_many(list(pop), tgt, H, W, 3.0, weight_mask=mask))
    assert np.max(np.abs(got - ref) / np.abs(ref)) <= 1e-5


def test_local_communicators(hip):
    """ggs_comm_init_local (ncclCommInitAll): one rank per listed device."""
    devs = (C.c_int32 * 1)(0)
    comms = (C.c_void_p * 1)()
    ggs._lib.check(ggs.lib.ggs_comm_init_local(1, devs, comms), "ggs_comm_init_local")
    n, r = C.c_int32(), C.c_int32()
    ggs._lib.check(ggs.lib.ggs_comm_size(comms[0], C.byref(n), C.byref(r)), "ggs_comm_size")
    assert (n.value, r.value) == (1, 0)
    ggs._lib.check(ggs.lib.ggs_comm_barrier(comms[0]), "ggs_comm_barrier")
    ggs.lib.ggs_comm_destroy(comms[0])
    bad = (C.c_int32 * 2)(0, 0)
    out2 = (C.c_void_p * 2)()
    with pytest.raises(ggs.GGSInputError):
        ggs._lib.check(ggs.lib.ggs_comm_init_local(2, bad, out2), "ggs_comm_init_local")


_FANOUT = r'''
import sys, numpy as np
sys.path[:0] = [{pkg!r}, {oracle!r}]
import ggs, ggs_oracle as O
H, W = 96, 80
pop = O.synthetic_population(37, 20, H, W, seed=4)
rng = np.random.default_rng(8)
tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
mask = rng.uniform(0.4, 1.0, (H, W)).astype(np.float32)
got = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask, n_devices=0)
np.save(sys.argv[1], got)
'''


def test_host_fanout_gathers_through_rccl(tmp_path):
    """The host API's multi-device fan-out returns the scalars with ONE RCCL
    all-gather + one D2H (north_star); GGS_FANOUT_RCCL=1 takes that path at one
    device: identical to the plain call, bit for bit."""
    script = _FANOUT.format(pkg=PKG, oracle=ORACLE)
    outs = []
    for force in ("0", "1"):
        path = str(tmp_path / f"fit{force}.npy")
        env = dict(os.environ, GGS_FANOUT_RCCL=force)
        subprocess.run([sys.executable, "-c", script, path], env=env, check=True, timeout=120)
        outs.append(np.load(path))
    np.testing.assert_array_equal(outs[0], outs[1])


def test_comm_argument_errors():
    h = C.c_void_p()
    idb = (C.c_uint8 * 128)()
    with pytest.raises(ggs.GGSInputError):
        ggs._lib.check(ggs.lib.ggs_comm_create(0, 2, 5, idb, C.byref(h)), "ggs_comm_create")
    with pytest.raises(ggs.GGSInputError):
        ggs._lib.check(ggs.lib.ggs_comm_wait(None, None, 0), "ggs_comm_wait")


@pytest.mark.parametrize("via", ["copy", "rccl"])
def test_device_ga_sharded_over_world1_comm_is_the_plain_ga(hip, via, monkeypatch):
    """ggs_ga_set_comm: breed all, evaluate this rank's shard, all-gather the
    fitness scalars — at world 1 the whole generation, bit-identical to the
    unsharded session (populations, fitness, best, curves).  "rccl" routes the
    single-rank gather through RCCL's in-place all-gather instead of the copy.
    set_comm also exchanges the sessions' fingerprints (here: with itself)."""
    if via == "rccl":
        monkeypatch.setenv("GGS_COMM_RCCL_SELF", "1")
    from ggs import ga
    from ggs.ga_device import DeviceGA
    H = W = 64
    rng = np.random.default_rng(5)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.4, 1.0, (H, W)).astype(np.float32)
    init = ga.new_population(24, 16, H, W, 3.0, 0.1, np.random.default_rng(2))
    cfg = dict(tour_k=2, elite_k=4, cxpb=0.3, mutpb=0.2, min_scale_splats=3.0, max_scale_splats=0.1,
               seed=9, schedule="cosine",
               mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0, "alpha": 25.0},
               mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0, "alpha": 2.0})
    res = []
    for shard in (False, True):
        d = DeviceGA(tgt, mask, init, **cfg)
        comm = ggs.RcclGather(0, rank=0, world=1) if shard else None
        if shard:
            d.set_comm(comm)
        d.run(1, 12, 12)
        res.append(d.read())
        d.close()
        if comm is not None:
            comm.close()
    a, b = res
    np.testing.assert_array_equal(a["population"], b["population"])
    np.testing.assert_array_equal(a["fitness"], b["fitness"])
    assert a["best_fit"] == b["best_fit"] and a["curves"] == b["curves"]


def test_configs3_sharded_over_eight_slots_equals_unsharded(hip, monkeypatch):
    """BASELINE configs[3] on one GPU: 1024^2, 1024 splats, pop 4096 split into the
    8 contiguous shards of an 8-rank job (``shard_bounds(4096, 8, r)``).  Each
    slot evaluates its shard straight into its offset of ONE gather buffer and
    runs its world-1 RCCL in-place all-gather there (the per-rank step of the
    8-GPU job, the device GA's layout).  The assembled vector equals the
    unsharded host-API ``ggs.fitness`` of all 4096 bit for bit, and the first and
    last candidates of two shards match the oracle (fitness.py:34-47)."""
    monkeypatch.setenv("GGS_COMM_RCCL_SELF", "1")       # world 1 through RCCL, not the copy kernel
    from ggs.parallel import shard_bounds
    H = W = 1024
    B, N, world = 4096, 1024, 8
    pop = O.synthetic_population(B, N, H, W, seed=33)
    rng = np.random.default_rng(34)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.405, 1.0, (H, W)).astype(np.float32)
    whole = ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask, device=0)     # unsharded

    g, t_d, m_d = (hip.DeviceArray.from_host(a) for a in (pop, tgt, mask))
    gath = hip.DeviceArray.from_host(np.full(B, np.nan, np.float32))
    st = hip.Stream()
    plan = ggs.TargetPlan(0, st.handle, t_d.ptr, m_d.ptr, ggs.GGS_FIT_WEIGHTED, 1.0, H, W)
    comms = [ggs.RcclGather(0, rank=0, world=1) for _ in range(world)]
    try:
        spans = [shard_bounds(B, world, r) for r in range(world)]
        assert [b1 - b0 for b0, b1 in spans] == [512] * world
        for r, (b0, b1) in enumerate(spans):
            slot = gath.ptr + 4 * b0
            plan.fitness_device(st.handle, g.ptr + 4 * 9 * N * b0, b1 - b0, N, 9, 3.0, slot)
            comms[r].allgather(st.handle, slot, slot, b1 - b0)                 # in place
        got = gath.to_host(st)
    finally:
        for c in comms:
            c.close()
        plan.close()
    np.testing.assert_array_equal(got, whole)
    picks = [spans[0][0], spans[0][1] - 1, spans[world - 1][0], spans[world - 1][1] - 1]
    ref = np.asarray(O.fitness_many([pop[i] for i in picks], tgt, H, W, 3.0, weight_mask=mask))
    assert np.max(np.abs(got[picks] - ref) / np.abs(ref)) <= 1e-5


# ---- loopback ranks: the sharded paths at world > 1 on one GPU ----------------------
def _loop_problem(H, N, P, seed):
    from ggs import ga
    rng = np.random.default_rng(seed)
    tgt = rng.uniform(0, 1, (H, H, 3)).astype(np.float32)
    mask = rng.uniform(0.4, 1.0, (H, H)).astype(np.float32)
    init = ga.new_population(P, N, H, H, 3.0, 0.1, np.random.default_rng(seed + 1))
    cfg = dict(tour_k=2, elite_k=8, cxpb=0.05, mutpb=0.05, min_scale_splats=3.0, max_scale_splats=0.1,
               seed=seed, schedule="cosine",
               mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0, "alpha": 25.0},
               mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0, "alpha": 2.0})
    return tgt, mask, init, cfg


def _set_comm_all(sessions, comms):
    """ggs_ga_set_comm on every rank at once (its fingerprint exchange is a host
    all-gather: one host thread per loopback rank); returns each rank's error."""
    import threading
    errs = [None] * len(sessions)

    def one(r):
        try:
            sessions[r].set_comm(comms[r])
        except Exception as e:  # noqa: BLE001 — reported per rank
            errs[r] = e
    ts = [threading.Thread(target=one, args=(r,)) for r in range(len(sessions))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    return errs


@pytest.mark.parametrize("H,N,P", [(512, 512, 32), (512, 256, 128)], ids=["shipped", "bench"])
@pytest.mark.parametrize("n", [2, 5, 7, 8])
def test_device_ga_loopback_ranks_equal_unsharded(hip, H, N, P, n):
    """The device GA's rank != 0 path (ggs_capi.cpp ga step: every rank breeds all
    P offspring with the same draws, rasterises its block [b0, b0+nb) of the
    P - E evaluated ones, per = ceil((P - E) / n), then one in-place all-gather of
    `per` scalars from offset rank*per) with n ranks on one GPU through a loopback
    group.  Shipped shape (config.py: 512^2, 512 splats, pop 32, elite 8 -> 24
    evaluated): n = 2 and 8 even shards, 5 uneven (5,5,5,5,4), 7 with an empty
    last rank (4 x 6 + 0).  Bench shape (pop 128 -> 120): 7 and 8 uneven.  Every
    rank's 20-generation trajectory (population, fitness, best, curves) equals
    the unsharded session's bit for bit (algorithm.py:123-141)."""
    from ggs.ga_device import DeviceGA
    from ggs.parallel import loopback_group
    tgt, mask, init, cfg = _loop_problem(H, N, P, seed=21)
    G = 20
    solo = DeviceGA(tgt, mask, init, **cfg)
    for g in range(1, G + 1):
        solo.step(g, G)
    ref = solo.read()
    solo.close()
    comms = loopback_group(0, n)
    ranks = [DeviceGA(tgt, mask, init, **cfg) for _ in range(n)]
    try:
        errs = _set_comm_all(ranks, comms)
        assert errs == [None] * n, errs
        for g in range(1, G + 1):
            for d in ranks:                  # lockstep: every rank once per generation
                d.step(g, G)
        for r, d in enumerate(ranks):
            st = d.read()
            np.testing.assert_array_equal(st["population"], ref["population"], err_msg=f"rank {r}")
            np.testing.assert_array_equal(st["fitness"], ref["fitness"], err_msg=f"rank {r}")
            assert st["best_fit"] == ref["best_fit"] and st["curves"] == ref["curves"], r
    finally:
        for d in ranks:
            d.close()
        for c in comms:
            c.close()


def test_device_ga_loopback_fingerprint_mismatch_fails_loudly(hip):
    """One rank with a different seed: every rank's ggs_ga_set_comm refuses
    (the shards would mix populations), naming the differing rank."""
    from ggs.ga_device import DeviceGA
    from ggs.parallel import loopback_group
    tgt, mask, init, cfg = _loop_problem(64, 16, 24, seed=3)
    n = 3
    comms = loopback_group(0, n)
    ranks = [DeviceGA(tgt, mask, init, **dict(cfg, seed=cfg["seed"] + (r == 2))) for r in range(n)]
    try:
        errs = _set_comm_all(ranks, comms)
        assert all(isinstance(e, ggs.GGSInputError) for e in errs), errs
        assert all("differs" in str(e) for e in errs), errs
    finally:
        for d in ranks:
            d.close()
        for c in comms:
            c.close()


def test_loopback_gather_out_of_lockstep_fails_loudly(hip):
    """A rank that issues its next device gather before every rank issued the
    current one fails (no silent reorder); a host gather with a rank missing
    times out with an error instead of hanging."""
    from ggs.parallel import loopback_group
    comms = loopback_group(0, 2)
    st = hip.Stream()
    buf = hip.DeviceArray((4,))
    try:
        comms[0].allgather(st.handle, buf.ptr, buf.ptr, 2)
        with pytest.raises(ggs.GGSInputError, match="lockstep"):
            comms[0].allgather(st.handle, buf.ptr, buf.ptr, 2)
        comms[1].allgather(st.handle, buf.ptr + 8, buf.ptr, 2)
        st.synchronize()
        os.environ["GGS_LOOPBACK_TIMEOUT_S"] = "1"
        with pytest.raises(ggs.GGSError, match="waited"):
            comms[0].barrier()
    finally:
        os.environ.pop("GGS_LOOPBACK_TIMEOUT_S", None)
        for c in comms:
            c.close()
