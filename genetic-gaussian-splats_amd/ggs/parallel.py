"""Multi-GPU evaluation: one process per GPU, contiguous candidate shards, one
all-gather of the fitness scalars.

The reference is single-device (render.py:4 hard-codes 'cuda'; SURVEY.md §5,
§8e).  Candidates are independent, so a generation of B candidates is split
into contiguous shards — rank r evaluates [b0, b1) on its own GPU with no data
exchange — and the only collective is one all-gather of B/world float32 scalars
per generation (``torch.distributed``, backend ``nccl`` = RCCL over xGMI on
MI355X; ``gloo`` in the CPU tests).  torch is used here purely as the
collective transport.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def shard_bounds(B: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous split of [0, B) — the same rule as the C library's
    multi-device fan-out (first B % world shards get one extra)."""
    base, rem = divmod(int(B), int(world))
    b0 = rank * base + min(rank, rem)
    return b0, b0 + base + (1 if rank < rem else 0)


def gather_shards(local: np.ndarray, B: int, group=None, device=None) -> np.ndarray:
    """All-gather every rank's contiguous fitness shard into the full [B] vector
    on every rank (one ``all_gather_into_tensor``; shards padded to ceil(B/world))."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    per = -(-int(B) // world)
    send = torch.zeros(per, dtype=torch.float32, device=device)
    if len(local):
        send[:len(local)] = torch.from_numpy(np.ascontiguousarray(local, np.float32)).to(send.device)
    recv = torch.empty(per * world, dtype=torch.float32, device=send.device)
    dist.all_gather_into_tensor(recv, send, group=group)
    full = recv.cpu().numpy()
    parts = []
    for r in range(world):
        b0, b1 = shard_bounds(B, world, r)
        parts.append(full[r * per:r * per + (b1 - b0)])
    return np.concatenate(parts) if parts else np.zeros(0, np.float32)


class ShardedFitness:
    """fitness_population over every rank of a process group.

    Each rank holds the same population (e.g. a GA driven with the same seed on
    every rank, or broadcast by rank 0), evaluates its shard on its local GPU
    through libggs.so and receives the full fitness vector.

    ``evaluate(G_shard) -> [b]`` defaults to :func:`ggs.fitness` with the target
    and mask given here; tests inject the oracle to exercise the gloo path on CPU.
    """

    def __init__(self, target, H: int, W: int, k_sigma: float = 3.0, weight_mask=None,
                 boost_only: bool = False, group=None, device=None,
                 evaluate: Optional[Callable[[np.ndarray], np.ndarray]] = None):
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device
        if evaluate is None:
            from . import api
            tgt, mask = api.as_f32(target), None if weight_mask is None else api.as_f32(weight_mask)

            def evaluate(G):
                return api.fitness(G, tgt, H, W, k_sigma, weight_mask=mask, boost_only=boost_only)
        self.evaluate = evaluate

    def __call__(self, population) -> np.ndarray:
        G = population if isinstance(population, np.ndarray) else \
            np.stack([np.asarray(p, np.float32) for p in population], 0)
        B = len(G)
        b0, b1 = shard_bounds(B, self.world, self.rank)
        local = np.asarray(self.evaluate(G[b0:b1]), np.float32) if b1 > b0 else np.zeros(0, np.float32)
        return gather_shards(local, B, self.group, self.device)


class RcclGather:
    """All-gather of each rank's fitness scalars over RCCL, issued by libggs on a
    HIP stream (``ggs_comm_*``, include/ggs.h) — the data-path collective of the
    sharded evaluation.  ``torch.distributed`` (any backend) only carries the
    128-byte communicator id from rank 0 to the others.

    ``allgather(stream, d_send, d_recv, count, overlap)`` takes device pointers;
    with ``overlap=True`` it returns a ticket and the gather runs on the
    communicator's own stream; ``wait(stream, ticket)`` joins it back (device-side).
    """

    def __init__(self, device: int, group=None):
        import ctypes as C
        import torch.distributed as dist
        from . import _lib
        _lib.preload_rccl()
        self._lib, self._C = _lib, C
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        idb = (C.c_uint8 * 128)()
        if self.rank == 0:
            _lib.check(_lib.lib.ggs_comm_unique_id(idb), "ggs_comm_unique_id")
        box = [bytes(idb)]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                   group=group)
        idb = (C.c_uint8 * 128).from_buffer_copy(box[0])
        h = C.c_void_p()
        _lib.check(_lib.lib.ggs_comm_create(int(device), self.world, self.rank, idb, C.byref(h)),
                   "ggs_comm_create")
        self.handle = h

    def allgather(self, stream: int, d_send: int, d_recv: int, count: int, overlap: bool = False) -> int:
        t = self._C.c_int64(-1)
        self._lib.check(self._lib.lib.ggs_comm_allgather(self.handle, stream, d_send, d_recv, int(count),
                                                         int(bool(overlap)), self._C.byref(t)),
                        "ggs_comm_allgather")
        return t.value

    def wait(self, stream: int, ticket: int) -> None:
        self._lib.check(self._lib.lib.ggs_comm_wait(self.handle, stream, int(ticket)), "ggs_comm_wait")

    def close(self) -> None:
        if self.handle:
            self._lib.lib.ggs_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
