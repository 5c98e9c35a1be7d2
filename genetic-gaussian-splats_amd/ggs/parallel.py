"""Multi-GPU evaluation: one process per GPU, contiguous candidate shards, one
all-gather of the fitness scalars.

The reference is single-device (render.py:4 hard-codes 'cuda'; SURVEY.md §5,
§8e).  Candidates are independent, so a generation of B candidates is split
into contiguous shards — rank r evaluates [b0, b1) on its own GPU with no data
exchange — and the only collective is one all-gather of the shards' float32
fitness scalars per generation over RCCL (xGMI), issued by libggs itself
(``ggs_comm_*``).  No PyTorch on this path: the 128-byte RCCL id travels
through a file rendezvous on the node (``file_rendezvous``).  ``ShardedFitness``
gathers through an ``RcclGather`` by default and keeps a ``torch.distributed``
transport (``gather_shards``) for callers that already run a process group.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
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
    """fitness_population (fitness.py:34-47) over every rank of a job.

    Each rank holds the same population (e.g. a GA driven with the same seed on
    every rank, or broadcast by rank 0), evaluates its contiguous shard on its
    local GPU through libggs.so and receives the full fitness vector.

    Transport, in this order: ``comm`` (an :class:`RcclGather`, or any object
    with ``rank``, ``world`` and ``allgather_host``); a ``torch.distributed``
    ``group`` (or the default group when one is initialised); otherwise an
    :class:`RcclGather` made here from the launcher's environment — the
    torch-free path (RCCL id through ``file_rendezvous``).

    ``evaluate(G_shard) -> [b]`` defaults to :func:`ggs.fitness` with the target
    and mask given here; tests inject the oracle to run the multi-rank logic on CPU.
    """

    def __init__(self, target, H: int, W: int, k_sigma: float = 3.0, weight_mask=None,
                 boost_only: bool = False, group=None, device=None,
                 evaluate: Optional[Callable[[np.ndarray], np.ndarray]] = None, comm=None):
        self.group, self.device, self.comm, self._own_comm = group, device, comm, False
        if comm is None and (group is not None or _torch_dist_initialized()):
            import torch.distributed as dist
            self.world = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
        else:
            if comm is None:
                from .api import device_index
                self.comm, self._own_comm = RcclGather(device_index(device)), True
            self.world, self.rank = int(self.comm.world), int(self.comm.rank)
        if evaluate is None:
            from . import api
            tgt, mask = api.as_f32(target), None if weight_mask is None else api.as_f32(weight_mask)

            def evaluate(G):
                return api.fitness(G, tgt, H, W, k_sigma, weight_mask=mask, boost_only=boost_only,
                                   device=device)
        self.evaluate = evaluate

    def __call__(self, population) -> np.ndarray:
        G = population if isinstance(population, np.ndarray) else \
            np.stack([np.asarray(p, np.float32) for p in population], 0)
        B = len(G)
        b0, b1 = shard_bounds(B, self.world, self.rank)
        local = np.asarray(self.evaluate(G[b0:b1]), np.float32) if b1 > b0 else np.zeros(0, np.float32)
        if self.comm is None:
            return gather_shards(local, B, self.group, self.device)
        per = -(-B // self.world)                  # equal slots: one all-gather, tail padded
        send = np.zeros(per, np.float32)
        send[:len(local)] = local
        return np.asarray(self.comm.allgather_host(send), np.float32).reshape(-1)[:B]

    def close(self) -> None:
        if self._own_comm and self.comm is not None:
            self.comm.close()
            self.comm = None


# ---- torch-free rendezvous -------------------------------------------------------
_RDZV_SEQ = [0]


def _torch_dist_initialized() -> bool:
    """A torch.distributed default group exists (checked without importing torch)."""
    d = sys.modules.get("torch.distributed")
    try:
        return bool(d is not None and d.is_available() and d.is_initialized())
    except Exception:  # noqa: BLE001 — a partially imported torch
        return False


def process_start_time(pid: int) -> Optional[float]:
    """Start time of process ``pid`` in seconds since the epoch (from /proc; 10-ms
    resolution), None when unknown."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        start_ticks = int(fields[19])                 # field 22 of stat(5)
        with open("/proc/stat") as f:
            btime = next(int(line.split()[1]) for line in f if line.startswith("btime"))
        return btime + start_ticks / os.sysconf("SC_CLK_TCK")
    except (OSError, ValueError, IndexError, StopIteration):
        return None


def launch_time() -> float:
    """When this launch began: the launcher (torchrun's agent or bench.py's spawner,
    the parent of every local rank) started before any rank wrote an id file, so a
    file older than it is left over from an earlier launch with the same key."""
    t = process_start_time(os.getppid())
    return (t - 0.05) if t is not None else 0.0


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
    MASTER_PORT, the run id and the elastic restart count — torchrun's agent
    survives a ``--max-restarts`` restart with the same pid, port and run id, so
    without the count a restarted rank could read the id file the crashed
    attempt left (newer than the agent, so ``launch_time`` does not reject it)."""
    k = os.environ.get("GGS_RDZV_KEY")
    if k:
        return k
    return "-".join([os.environ.get("TORCHELASTIC_RUN_ID", "run"), os.environ.get("MASTER_PORT", "0"),
                     str(os.getppid()), "a" + os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")])


def file_rendezvous(rank: int, world: int, make_id, key: Optional[str] = None,
                    timeout_s: float = 300.0, directory: Optional[str] = None) -> bytes:
    """Carry the 128-byte RCCL id from rank 0 to the other ranks of THIS node
    without a process group: rank 0 writes it atomically (tmp + rename) to a file
    named by ``key`` and a per-process sequence number (the n-th communicator
    every rank makes); the others poll for it and accept only a file written after
    the launch began (``launch_time``), so an id left behind by an earlier launch
    that crashed before rank 0 could remove it is never read (an elastic restart
    under the same agent is told apart by the restart count in
    ``rendezvous_key``, not by the file's age).  Rank 0 removes the file
    once the communicator exists (all ranks have read it: RCCL's init is
    collective).  Single node only — the scope of north_star's 8-GPU sharding."""
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
    fresh_after = launch_time()
    while True:
        try:
            with open(path, "rb") as f:
                idb = f.read()
                mtime = os.fstat(f.fileno()).st_mtime
            if len(idb) == 128 and mtime >= fresh_after:   # not a crashed launch's left-over
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
        self.handle = None
        _lib.preload_rccl()
        self._lib, self._C = _lib, C
        if group is None and rank is None and world is None and _torch_dist_initialized():
            import torch.distributed as dist     # an existing process group carries the id
            group = dist.group.WORLD
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
            lw = os.environ.get("LOCAL_WORLD_SIZE")
            if world is None and self.world > 1 and lw is not None and int(lw) != self.world:
                raise RuntimeError(
                    f"RcclGather: WORLD_SIZE={self.world} spans more than this node "
                    f"(LOCAL_WORLD_SIZE={lw}); the file rendezvous is node-local — pass a "
                    f"torch.distributed `group` (or initialise the default process group) instead")

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

    def info(self):
        """(ranks, rank, device) as RCCL itself reports them (ncclCommCount,
        ncclCommUserRank, ncclCommCuDevice) — not the values this object was asked for."""
        n, r, d = self._C.c_int32(0), self._C.c_int32(0), self._C.c_int32(0)
        self._lib.check(self._lib.lib.ggs_comm_info(self.handle, self._C.byref(n), self._C.byref(r),
                                                    self._C.byref(d)), "ggs_comm_info")
        return n.value, r.value, d.value

    def close(self) -> None:
        if self.handle:
            self._lib.lib.ggs_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def loopback_group(device: int, n: int) -> list:
    """n communicators on ONE device of this process acting as ranks 0..n-1 of one
    job (``ggs_comm_init_loopback``; a test rig, no RCCL): the sharded code paths
    (rank != 0, uneven and empty shards, the GA's fingerprint exchange) run on a
    one-GPU box.  Device all-gathers must be issued in lockstep (every rank once
    per gather): the last rank's call enqueues every shard copy, so a rank's
    d_recv is defined on its stream only after all ranks have called for that
    gather; a HIP failure during that enqueue makes the group unusable (every later
    call fails).  Host all-gathers need one host thread per rank.  Each returned
    object has RcclGather's interface."""
    from . import _lib
    arr = (C.c_void_p * int(n))()
    _lib.check(_lib.lib.ggs_comm_init_loopback(int(device), int(n), arr), "ggs_comm_init_loopback")
    out = []
    for r in range(int(n)):
        g = RcclGather.__new__(RcclGather)
        g._lib, g._C, g.rank, g.world, g.handle = _lib, C, r, int(n), C.c_void_p(arr[r])
        out.append(g)
    return out

