"""CPU stand-ins for the GPU side of the multi-rank path (test infrastructure).

* ``PipeMesh`` / ``PipeComm``: an in-memory all-gather between rank processes
  over multiprocessing pipes, with the interface of ``ggs.RcclGather``
  (``rank``, ``world``, ``allgather``, ``wait``, ``allgather_host``, ``barrier``,
  ``close``).  Its 128-byte id still travels through the REAL
  ``ggs.parallel.file_rendezvous`` (rank 0 writes, the others poll), and every
  rank checks that it received rank 0's bytes.  Each message carries
  (communicator sequence number, call number, kind), so two ranks that issue
  their collectives in a different order or a different number of times fail
  loudly instead of pairing the wrong calls.  Like an in-stream RCCL gather,
  ``allgather`` only posts this rank's part and returns; the peers' parts are
  received when a host collective (``barrier`` / ``allgather_host``) or a full
  in-flight window drains the posted calls of every communicator in issue order
  (they share the pipes).  ``stall=(rank, n)`` makes
  that rank block forever in its n-th gather before posting it (a rank that
  never issues a collective the others wait on).
* ``install_fake_gpu``: ``ggs`` / ``ggs.hip`` modules whose device memory is a
  registry of numpy arrays, so ``bench.run()`` executes its whole distributed
  control flow (rendezvous, ramps, timed passes, max over ranks, shard check,
  JSON line) on CPU.  The stand-in fitness of a candidate is the float32 sum of
  its genome; nothing here is the product.
"""
from __future__ import annotations

import itertools
import os
import sys
import types

import numpy as np

from conftest import PKG

TIMEOUT_S = 60.0


def real_parallel():
    """ggs/parallel.py itself, loaded from its file (the stand-in ``ggs`` package
    of ``install_fake_gpu`` would shadow ``ggs.parallel``)."""
    import importlib.util
    m = sys.modules.get("_ggs_parallel_real")
    if m is None:
        spec = importlib.util.spec_from_file_location("_ggs_parallel_real",
                                                      os.path.join(PKG, "ggs", "parallel.py"))
        m = importlib.util.module_from_spec(spec)
        sys.modules["_ggs_parallel_real"] = m
        spec.loader.exec_module(m)
    return m


class PipeMesh:
    """One duplex pipe per rank pair, made in the parent before the fork."""

    def __init__(self, world: int, ctx):
        self.world = world
        self.ends = {}
        for a, b in itertools.combinations(range(world), 2):
            ea, eb = ctx.Pipe(duplex=True)
            self.ends[(a, b)], self.ends[(b, a)] = ea, eb

    def peer(self, rank: int, q: int):
        return self.ends[(rank, q)]


class PipeComm:
    _seq = itertools.count()              # n-th communicator this process made

    WINDOW = 8                            # posted gathers before a forced drain
    _pending = []                         # posted, not yet received (issue order, all communicators)
    _gathers = itertools.count()          # gathers this process entered (all communicators)

    def __init__(self, mesh: PipeMesh, rank: int, world: int, log=None, corrupt=False, key=None,
                 stall=None):
        file_rendezvous = real_parallel().file_rendezvous
        self.mesh, self.rank, self.world, self.log = mesh, rank, world, log
        self.corrupt, self.stall = corrupt, stall
        self.cid = next(PipeComm._seq)
        self.calls = 0
        self.tickets = {}
        self.pending = PipeComm._pending      # one queue: every communicator shares the pipes
        idb = file_rendezvous(rank, world, lambda: os.urandom(128), key)
        ids = self._exchange("id", np.frombuffer(idb, np.uint8).copy())
        assert all(bytes(x) == bytes(ids[0]) for x in ids), "ranks received different communicator ids"
        self.id = bytes(idb)
        if log is not None:
            log.setdefault("comms", []).append({"cid": self.cid, "id": self.id.hex()[:16]})

    def _post(self, kind: str, payload: np.ndarray, done) -> None:
        """Send this rank's payload to every peer now; ``done(parts)`` runs when
        the call is drained."""
        tag = (self.cid, self.calls, kind)
        self.calls += 1
        for q in range(self.world):
            if q != self.rank:
                self.mesh.peer(self.rank, q).send((tag, payload))
        self.pending.append((tag, payload, done))

    def _drain(self) -> None:
        """Receive every posted call's parts from the peers, in issue order."""
        while self.pending:
            tag, payload, done = self.pending.pop(0)
            out = [None] * self.world
            out[self.rank] = payload
            for q in range(self.world):
                if q == self.rank:
                    continue
                c = self.mesh.peer(self.rank, q)
                if not c.poll(TIMEOUT_S):
                    raise TimeoutError(f"rank {self.rank}: no {tag[2]} from rank {q} (call {tag})")
                rtag, data = c.recv()
                if rtag != tag:
                    raise AssertionError(f"rank {self.rank} issued {tag} but rank {q} issued {rtag}")
                out[q] = data
            done(out)

    def _exchange(self, kind: str, payload: np.ndarray):
        """Every rank's payload, in rank order (a blocking call: drains first)."""
        box = []
        self._post(kind, payload, box.append)
        self._drain()
        return box[0]

    # ---- the RcclGather interface --------------------------------------------------
    def allgather(self, stream, d_send, d_recv, count, overlap=False):
        if self.stall is not None and self.stall[0] == self.rank and next(PipeComm._gathers) == self.stall[1]:
            import time
            time.sleep(3600)                          # never issues this gather
        send = MEM[d_send].reshape(-1)[:count].copy()

        def done(parts):
            recv = MEM[d_recv].reshape(-1)
            for r, p in enumerate(parts):
                recv[r * count:(r + 1) * count] = p
            if self.corrupt:
                recv[self.rank * count] += 1.0
        self._post("gather", send, done)
        if len(self.pending) >= self.WINDOW:
            self._drain()
        if self.log is not None:
            g = self.log.setdefault("gathers", {})
            g[str(self.cid)] = g.get(str(self.cid), 0) + 1
            self.log["gather_count"] = int(count)
        if overlap:
            t = len(self.tickets)
            self.tickets[t] = True
            return t
        return -1

    def wait(self, stream, ticket):
        if ticket >= 0:
            self._drain()
            assert self.tickets.pop(ticket), "wait on an unknown ticket"

    def allgather_host(self, values):
        v = np.ascontiguousarray(values, np.float32).reshape(-1)
        return np.stack(self._exchange("host", v), 0)

    def barrier(self):
        self._exchange("barrier", np.zeros(0, np.float32))

    def info(self):
        """(ranks, rank, device) as RCCL reports them: this rank's device is its LOCAL_RANK."""
        return self.world, self.rank, int(self.log.get("device", -1)) if self.log is not None else -1

    def close(self):
        pass


# ---- fake device memory + ggs modules for bench.run() -------------------------------
MEM = {}
_ptrs = itertools.count(0x1000, 0x1000)


class _DeviceArray:
    def __init__(self, shape, dtype=np.float32):
        self.shape = tuple(np.atleast_1d(shape)) if not isinstance(shape, tuple) else shape
        self.a = np.zeros(self.shape, dtype)
        self.ptr = next(_ptrs)
        MEM[self.ptr] = self.a

    @classmethod
    def from_host(cls, a):
        d = cls(a.shape, a.dtype)
        d.a[...] = a
        return d

    def to_host(self, stream=None):
        return self.a.copy()


class _Stream:
    _h = itertools.count(1)

    def __init__(self):
        self.handle = next(self._h)

    def synchronize(self):
        pass


def install_fake_gpu(mesh, rank, world, log, slow_rank=None, corrupt=False, stall=None):
    """Put stand-in ``ggs`` and ``ggs.hip`` modules in sys.modules."""
    import time

    hip = types.ModuleType("ggs.hip")
    hip.DeviceArray, hip.Stream = _DeviceArray, _Stream
    hip.set_device = lambda d: log.__setitem__("device", int(d))
    hip.synchronize = lambda: None

    def memcpy_d2h_async(host, ptr, nbytes, stream):
        host.reshape(-1).view(np.uint8)[:nbytes] = MEM[ptr].reshape(-1).view(np.uint8)[:nbytes]
    hip.memcpy_d2h_async = memcpy_d2h_async

    class TargetPlan:
        def __init__(self, device, stream, d_target, d_mask, mode, beta, H, W):
            log["plan"] = [int(device), int(H), int(W), int(mode)]

        def fitness_device(self, stream, d_genomes, B, N, Cc, k_sigma, d_out):
            g = MEM[d_genomes].reshape(-1, N, Cc)
            assert g.shape[0] == B, (g.shape, B)
            MEM[d_out].reshape(-1)[:B] = g.reshape(B, -1).sum(1, dtype=np.float32)
            log.setdefault("batches", set()).add(int(B))
            if slow_rank == rank:
                time.sleep(0.001)

    prof = {}
    ggs = types.ModuleType("ggs")
    ggs.hip = hip
    ggs.GGS_FIT_WEIGHTED = 1
    ggs.LIB_PATH = os.path.join(PKG, "libggs.so")    # the built library (bench hashes it)
    ggs.ensure_init = lambda: max(world, 1)
    ggs.select_devices = lambda ids: log.__setitem__("selected", list(ids))
    ggs.TargetPlan = TargetPlan
    TargetPlan.close = lambda self: None

    def fitness_device(dev, st, d_gen, B, N, Cc, d_t, d_m, mode, beta, H, W, k, d_out):
        TargetPlan(dev, st, d_t, d_m, mode, beta, H, W).fitness_device(st, d_gen, B, N, Cc, k, d_out)
    ggs.fitness_device = fitness_device
    ggs.fitness = lambda G, tgt, H, W, k, weight_mask=None, device=0: \
        np.asarray(G, np.float32).reshape(len(G), -1).sum(1, dtype=np.float32)
    ggs.RcclGather = lambda local_rank: PipeComm(mesh, rank, world, log, corrupt, stall=stall)
    ggs.profile_reset = prof.clear
    ggs.profile_enable = lambda on: None
    ggs.profile_read = lambda k: (0.1, 1)
    ggs.encode = lambda G: np.asarray(G, np.float32)
    ggs.runtime_info = lambda: {"hip": "/fake/rocm/lib/libamdhip64.so.7", "hip_version": 1,
                                "rccl": "/fake/rocm/lib/librccl.so.1", "rccl_version": 1, "same_tree": True}

    def preprocess(G, H, W, k):
        n = int(np.prod(G.shape[:-1]))
        z = np.zeros(n, np.int32)
        return {"x0": z, "x1": z + 3, "y0": z, "y1": z + 3}
    ggs.preprocess = preprocess
    ggs.parallel = real_parallel()          # rendezvous_key for the heartbeat files
    sys.modules["ggs"], sys.modules["ggs.hip"], sys.modules["ggs.parallel"] = ggs, hip, ggs.parallel
    return ggs
