"""The multi-GPU data-path collective through the C ABI:
``ggs_comm_*`` all-gathers per-rank fitness scalars over RCCL on a HIP stream,
in-stream or overlapped on the communicator's own stream.  One GPU here, so a
world-1 communicator (rank 0's id carried over a gloo process group, as
``ggs.RcclGather`` does at any world size); the N > 1 sharding logic is covered
on CPU by tests/test_dist_gloo.py and run at N = 2..8 by bench.py.
"""
from __future__ import annotations

import numpy as np
import pytest

import ggs
import ggs_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world1():
    import socket

    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [False, True])
def test_rccl_allgather_returns_every_shard(world1, overlap):
    import torch
    dev = torch.device("cuda", 0)
    comm = ggs.RcclGather(0)
    st = torch.cuda.current_stream(dev).cuda_stream
    try:
        for count in (1, 128, 4099):
            send = torch.arange(count, dtype=torch.float32, device=dev) * 0.5 - 3.0
            recv = torch.full((count * comm.world,), float("nan"), device=dev)
            t = comm.allgather(st, send.data_ptr(), recv.data_ptr(), count, overlap=overlap)
            assert (t >= 0) == overlap
            comm.wait(st, t)
            torch.cuda.synchronize(dev)
            assert torch.equal(recv[comm.rank * count:(comm.rank + 1) * count], send)
    finally:
        comm.close()


def test_sharded_fitness_through_rccl_matches_oracle(world1):
    """bench.py's step: fused fitness of this rank's candidates into a ring slot,
    overlapped gather, join — the gathered vector equals the oracle's fitness."""
    import torch
    dev = torch.device("cuda", 0)
    H = W = 64
    B, N = 6, 12
    pop = O.synthetic_population(B, N, H, W, seed=7)
    rng = np.random.default_rng(3)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = rng.uniform(0.4, 1.0, (H, W)).astype(np.float32)
    g = torch.from_numpy(pop).to(dev)
    t_d, m_d = torch.from_numpy(tgt).to(dev), torch.from_numpy(mask).to(dev)
    out = torch.empty(B, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    comm = ggs.RcclGather(0)
    try:
        plan = ggs.TargetPlan(0, st, t_d.data_ptr(), m_d.data_ptr(), ggs.GGS_FIT_WEIGHTED, 1.0, H, W)
        plan.fitness_device(st, g.data_ptr(), B, N, 9, 3.0, out.data_ptr())
        full = torch.empty(B * comm.world, device=dev)
        comm.wait(st, comm.allgather(st, out.data_ptr(), full.data_ptr(), B, overlap=True))
        got = full.cpu().numpy()[:B]
    finally:
        comm.close()
    ref = np.asarray(O.fitness_many(list(pop), tgt, H, W, 3.0, weight_mask=mask))
    assert np.max(np.abs(got - ref) / np.abs(ref)) <= 1e-5


def test_comm_argument_errors():
    import ctypes as C
    h = C.c_void_p()
    idb = (C.c_uint8 * 128)()
    with pytest.raises(ggs.GGSInputError):
        ggs._lib.check(ggs.lib.ggs_comm_create(0, 2, 5, idb, C.byref(h)), "ggs_comm_create")
    with pytest.raises(ggs.GGSInputError):
        ggs._lib.check(ggs.lib.ggs_comm_wait(None, None, 0), "ggs_comm_wait")


@pytest.mark.parametrize("via", ["copy", "rccl"])
def test_device_ga_sharded_over_world1_comm_is_the_plain_ga(world1, via, monkeypatch):
    """ggs_ga_set_comm: breed all, evaluate this rank's shard, all-gather the
    fitness scalars — at world 1 the whole generation, bit-identical to the
    unsharded session (populations, fitness, best, curves).  "rccl" routes the
    single-rank gather through RCCL's in-place all-gather instead of the copy."""
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
        comm = ggs.RcclGather(0) if shard else None
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
