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
