"""Multi-GPU evaluation: one process per GPU, contiguous candidate shards, one
all-gather of the fitness scalars.

The reference is single-device (render.py:4 hard-codes 'cuda'; SURVEY.md §5,
§8e).  Candidates are independent, so a generation of B candidates is split
into contiguous shards — rank r evaluates [b0, b1) on its own GPU with no data
exchange — and the only collective is one all-gather of the shards' float32
fitness scalars per generation over RCCL (xGMI), issued by libggs itself
(``ggs_comm_*``).  No PyTorch on this path: the 128-byte RCCL id travels
through a file rendezvous on the node (``file_rendezvous``).  ``ShardedFitness``
and ``gather_shards`` keep a ``torch.distributed`` transport for callers that
already run a process group (the CPU tests use ``gloo``).
"""
from __future__ import annotations

import ctypes as C
import os
import tempfile
import time
from typing import Callable, Optional, Tuple

import numpy as np


def shard_bounds(B: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous split of [0, B) into slots of ceil(B/world) (the last shards
    shorter or empty) — the same rule as the C library's multi-device fan-out and
    the device GA's shards, so the slots meet in one in-place all-gather."""
    per = -(-int(B) // int(world))
    b0 = min(int(B), rank * per)
    return b0, min(int(B), b0 + per)


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
    return recv.cpu().numpy()[:int(B)]            # slot r holds [r*per, r*per + per) ∩ [0, B)


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


# ---- torch-free rendezvous -------------------------------------------------------
_RDZV_SEQ = [0]


def launch_env():
    """(rank, world, local_rank) from the launcher's environment (torchrun, or
    bench.py's own spawner): RANK / WORLD_SIZE / LOCAL_RANK, defaults 0 / 1 / rank."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, world, int(os.environ.get("LOCAL_RANK", str(rank)))


def rendezvous_key() -> str:
    """Names one launch of one job on this node: every rank of it computes the
    same key.  ``GGS_RDZV_KEY`` overrides; otherwise the launcher's parent pid
    (torchrun's agent or bench.py's spawner starts every local rank) with
    MASTER_PORT and the run id."""
    k = os.environ.get("GGS_RDZV_KEY")
    if k:
        return k
    return "-".join([os.environ.get("TORCHELASTIC_RUN_ID", "run"), os.environ.get("MASTER_PORT", "0"),
                     str(os.getppid())])


def file_rendezvous(rank: int, world: int, make_id, key: Optional[str] = None,
                    timeout_s: float = 300.0, directory: Optional[str] = None) -> bytes:
    """Carry the 128-byte RCCL id from rank 0 to the other ranks of THIS node
    without a process group: rank 0 writes it atomically (tmp + rename) to a file
    named by ``key`` and a per-process sequence number (the n-th communicator
    every rank makes); the others poll for it.  Rank 0 removes the file in
    ``release_rendezvous`` once the communicator exists (all ranks have read it:
    RCCL's init is collective).  Single node only — the scope of north_star's
    8-GPU sharding."""
    seq = _RDZV_SEQ[0]
    _RDZV_SEQ[0] += 1
    d = directory or os.environ.get("GGS_RDZV_DIR") or tempfile.gettempdir()
    path = os.path.join(d, f"ggs-rdzv-{key or rendezvous_key()}-{seq}-w{world}.id")
    if rank == 0:
        idb = bytes(make_id())
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(idb)
        os.replace(tmp, path)
        return idb
    t0 = time.monotonic()
    while True:
        try:
            with open(path, "rb") as f:
                idb = f.read()
            if len(idb) == 128:
                return idb
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout_s:
            raise TimeoutError(f"rank {rank}: no RCCL id from rank 0 at {path} after {timeout_s:.0f} s")
        time.sleep(0.01)


def _rendezvous_path_of_last(key: Optional[str], world: int, directory: Optional[str] = None) -> str:
    d = directory or os.environ.get("GGS_RDZV_DIR") or tempfile.gettempdir()
    return os.path.join(d, f"ggs-rdzv-{key or rendezvous_key()}-{_RDZV_SEQ[0] - 1}-w{world}.id")


class RcclGather:
    """All-gather of each rank's fitness scalars over RCCL, issued by libggs on a
    HIP stream (``ggs_comm_*``, include/ggs.h) — the data-path collective of the
    sharded evaluation.  The 128-byte communicator id goes from rank 0 to the
    others through ``file_rendezvous`` (no PyTorch), or through ``group`` when a
    ``torch.distributed`` process group is passed.

    ``allgather(stream, d_send, d_recv, count, overlap)`` takes device pointers;
    with ``overlap=True`` it returns a ticket and the gather runs on the
    communicator's own stream; ``wait(stream, ticket)`` joins it back (device-side).
    ``barrier()`` and ``allgather_host(values)`` are host-side collectives over
    the same communicator (timings, checks).
    """

    def __init__(self, device: int, group=None, rank: Optional[int] = None,
                 world: Optional[int] = None, key: Optional[str] = None):
        from . import _lib
        _lib.preload_rccl()
        self._lib, self._C = _lib, C
        if group is not None:
            import torch.distributed as dist
            self.world = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
            idb = (C.c_uint8 * 128)()
            if self.rank == 0:
                _lib.check(_lib.lib.ggs_comm_unique_id(idb), "ggs_comm_unique_id")
            box = [bytes(idb)]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0), group=group)
            raw = box[0]
        else:
            r, w, _ = launch_env()
            self.rank = r if rank is None else int(rank)
            self.world = w if world is None else int(world)

            def make_id():
                b = (C.c_uint8 * 128)()
                _lib.check(_lib.lib.ggs_comm_unique_id(b), "ggs_comm_unique_id")
                return bytes(b)
            raw = make_id() if self.world == 1 else file_rendezvous(self.rank, self.world, make_id, key)
        idb = (C.c_uint8 * 128).from_buffer_copy(raw)
        h = C.c_void_p()
        _lib.check(_lib.lib.ggs_comm_create(int(device), self.world, self.rank, idb, C.byref(h)),
                   "ggs_comm_create")
        self.handle = h
        if group is None and self.rank == 0 and self.world > 1:   # every rank joined: the id file is spent
            try:
                os.unlink(_rendezvous_path_of_last(key, self.world))
            except OSError:
                pass

    def allgather(self, stream: int, d_send: int, d_recv: int, count: int, overlap: bool = False) -> int:
        t = self._C.c_int64(-1)
        self._lib.check(self._lib.lib.ggs_comm_allgather(self.handle, stream, d_send, d_recv, int(count),
                                                         int(bool(overlap)), self._C.byref(t)),
                        "ggs_comm_allgather")
        return t.value

    def wait(self, stream: int, ticket: int) -> None:
        self._lib.check(self._lib.lib.ggs_comm_wait(self.handle, stream, int(ticket)), "ggs_comm_wait")

    def allgather_host(self, values) -> np.ndarray:
        """Every rank's float32 ``values`` (same length everywhere) → [world, len]."""
        v = np.ascontiguousarray(values, np.float32).reshape(-1)
        out = np.empty((self.world, v.size), np.float32)
        f32p = self._C.POINTER(self._C.c_float)
        self._lib.check(self._lib.lib.ggs_comm_allgather_host(self.handle, v.ctypes.data_as(f32p),
                                                              out.ctypes.data_as(f32p), v.size),
                        "ggs_comm_allgather_host")
        return out

    def barrier(self) -> None:
        self._lib.check(self._lib.lib.ggs_comm_barrier(self.handle), "ggs_comm_barrier")

    def close(self) -> None:
        if self.handle:
            self._lib.lib.ggs_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
