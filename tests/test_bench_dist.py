"""bench.py's N > 1 orchestration, executed on CPU at world 2 (no GPU).

Each rank is a forked process that runs ``bench.main()`` exactly as under
``torch.distributed.run`` (RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE in
the environment), with the GPU side replaced by ``tests/_fakes.py``: device
memory is a numpy registry and each communicator is an in-memory all-gather
over pipes whose id is carried by the real ``ggs.parallel.file_rendezvous``.
What runs for real is bench.py's control flow: four communicators per rank
made in the same sequence, the ramps, the timed passes (rank 1 is made slower,
so only the max over ranks keeps the pass counts equal — a mismatch pairs the
wrong collectives and fails), the shard check, and rank 0's JSON line.
The sharded evaluation of ``ggs.parallel.ShardedFitness`` is covered the same
way (torch-free comm, world 2, oracle as the evaluator).
"""
from __future__ import annotations

import contextlib
import json
import multiprocessing as mp
import os
import sys

import numpy as np
import pytest

from conftest import ORACLE, PKG, REPO

sys.path.insert(0, REPO)


def _rank_main(rank, world, mesh, argv, out_dir, slow_rank, corrupt, stall=None):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT="29555",
                      GGS_RDZV_DIR=out_dir, GGS_RDZV_KEY="bench-dist-test")
    sys.stderr = open(os.path.join(out_dir, f"stderr{rank}.txt"), "w", buffering=1)
    import _fakes
    log = {}
    _fakes.install_fake_gpu(mesh, rank, world, log, slow_rank=slow_rank, corrupt=corrupt, stall=stall)
    import bench
    rc = 0
    with open(os.path.join(out_dir, f"stdout{rank}.txt"), "w") as f, contextlib.redirect_stdout(f):
        try:
            bench.main(argv)
        except AssertionError as e:
            log["assertion"] = str(e)
            rc = 3
    log["batches"] = sorted(log.get("batches", ()))
    with open(os.path.join(out_dir, f"log{rank}.json"), "w") as f:
        json.dump(log, f)
    os._exit(rc)


def _run_world(tmp_path, argv, world=2, slow_rank=1, corrupt=False, stall=None):
    import _fakes
    ctx = mp.get_context("fork")
    mesh = _fakes.PipeMesh(world, ctx)
    procs = [ctx.Process(target=_rank_main, args=(r, world, mesh, argv, str(tmp_path), slow_rank, corrupt, stall))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        if p.is_alive():
            p.kill()
            raise TimeoutError("a rank hung")
    if stall is not None:
        return [p.exitcode for p in procs], None, None
    logs = [json.load(open(tmp_path / f"log{r}.json")) for r in range(world)]
    out0 = (tmp_path / "stdout0.txt").read_text().strip().splitlines()
    return [p.exitcode for p in procs], logs, out0


FAST = ["--steps", "3", "--warmup", "2", "--min-time", "0.02", "--ramp-ms", "1", "--no-cpu-baseline"]


def test_bench_world2_orchestration(tmp_path):
    codes, logs, out0 = _run_world(tmp_path, ["--gpus", "2"] + FAST)
    assert codes == [0, 0], logs
    # four communicators per rank, made in the same sequence from the same ids
    assert [len(lg["comms"]) for lg in logs] == [4, 4]
    assert logs[0]["comms"] == logs[1]["comms"]
    # the same collectives, the same number of times, on every communicator
    assert logs[0]["gathers"] == logs[1]["gathers"] and sum(logs[0]["gathers"].values()) > 0
    assert [lg["device"] for lg in logs] == [0, 1] and [lg["selected"] for lg in logs] == [[0], [1]]
    assert all(lg["batches"] == [128] for lg in logs) and logs[0]["gather_count"] == 128
    assert "assertion" not in logs[0] and "assertion" not in logs[1]      # shard_ok held
    assert len(out0) == 1
    line = json.loads(out0[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["rccl_ranks"] == 2 and line["config"]["global_batch"] == 256
    assert line["config"]["fitness_gather"] == "rccl" and line["config"]["pop_per_gpu"] == 128
    assert line["timing"]["passes"] >= 1 and line["value"] > 0
    assert line["roofline"]["binding"] == "valu" and line["roofline"]["bound"] == "valu"
    pe = line["plan_excluded"]
    assert pe["device_api_unplanned_value"] > 0 and pe["plan_build_ms"] >= 0
    assert not (tmp_path / "stdout1.txt").read_text().strip()               # rank 1 prints nothing


@pytest.mark.parametrize("world", [4, 8])
def test_bench_world_n_orchestration(tmp_path, world):
    """The same control flow at the driver's larger worlds: every rank makes its
    four communicators from the same ids, issues the same collectives, and rank 0
    alone prints one line with n_gpus = world and global_batch = 128 * world."""
    codes, logs, out0 = _run_world(tmp_path, ["--gpus", str(world)] + FAST, world=world)
    assert codes == [0] * world, logs
    assert all(lg["comms"] == logs[0]["comms"] and lg["gathers"] == logs[0]["gathers"] for lg in logs)
    assert [lg["device"] for lg in logs] == list(range(world))
    line = json.loads(out0[0])
    assert line["n_gpus"] == world and line["config"]["global_batch"] == 128 * world
    assert line["config"]["rccl_ranks"] == world and len(out0) == 1
    # rank -> device from each rank's communicator (RCCL's own report), gathered
    assert line["config"]["rank_devices"] == [[r, r] for r in range(world)]
    assert line["runtime"]["same_tree"] is True


def test_bench_world2_strong_scaling_splits_configs3(tmp_path):
    """--config 1024x8 (configs[3]): one population of 4096 split 2048 per rank,
    2048 fitness scalars per rank in each gather, global_batch 4096."""
    codes, logs, out0 = _run_world(tmp_path, ["--gpus", "2", "--config", "1024x8"] + FAST)
    assert codes == [0, 0], logs
    assert all(lg["batches"] == [2048] for lg in logs)
    assert logs[0]["gather_count"] == 2048 and logs[0]["plan"] == [0, 1024, 1024, 1]
    line = json.loads(out0[0])
    assert line["scaling"] == "strong" and line["n_gpus"] == 2
    assert line["config"]["global_batch"] == 4096 and line["config"]["pop_per_gpu"] == 2048


@pytest.mark.parametrize("stall_at", [0, 9])
def test_bench_world2_stalled_gather_fails_loudly_naming_the_rank(tmp_path, stall_at):
    """Rank 1 never issues one fitness gather (its stand-in communicator blocks
    forever in that call: gather 0 sits in the warm-up, gather 9 in the first timed
    pass).  Rank 0 issues past it and waits in the pass's barrier.  Each rank's
    watchdog fires at its phase deadline (floor 2 s here), every rank exits with
    WATCHDOG_EXIT well before the stand-in transport's own 60 s timeout, and both
    name rank 1 from the heartbeat files, with phase, step, stream and the
    collectives issued on stderr."""
    import time
    import bench
    t0 = time.monotonic()
    codes, _, _ = _run_world(tmp_path, ["--gpus", "2", "--watchdog-floor-s", "2"] + FAST,
                             stall=(1, stall_at))
    took = time.monotonic() - t0
    assert codes == [bench.WATCHDOG_EXIT] * 2
    assert took < 30, took
    for r in range(2):
        err = (tmp_path / f"stderr{r}.txt").read_text()
        assert f"bench.py watchdog: rank {r}: phase" in err, err
        assert "stalled rank(s): [1]" in err, err
        assert "rank 0: phase" in err and "rank 1: phase" in err and "issued" in err, err
    assert "gather" not in (tmp_path / "stdout0.txt").read_text()            # no JSON line


def test_watchdog_names_frozen_or_lagging_ranks():
    import bench
    now = 1000.0
    hb = {r: {"wall": now, "issued_total": 12} for r in range(4)}
    assert bench.Watchdog.stalled(hb, now, 5.0)[0] == []                       # a device hang
    hb[2]["issued_total"] = 9
    assert bench.Watchdog.stalled(hb, now, 5.0)[0] == [2]
    hb[3] = None
    assert bench.Watchdog.stalled(hb, now, 5.0)[0] == [3]
    hb[3] = {"wall": now - 60, "issued_total": 12}
    assert bench.Watchdog.stalled(hb, now, 5.0)[0] == [3]


def test_stream_accounting_refuses_shared_queues():
    import bench
    a = bench.stream_accounting(4, True, "rccl", 8)
    assert a["collective_streams"] == 5 and a["communicator_streams"] == 1 and a["ok"]
    assert bench.stream_accounting(4, True, "rccl-overlap", 8)["collective_streams"] == 4
    assert not bench.stream_accounting(8, True, "rccl", 8)["ok"]
    w1 = bench.stream_accounting(4, False, "rccl", 4)
    assert w1["collective_streams"] == 0 and w1["communicators"] == 0 and w1["ok"]


def test_bench_refuses_more_collective_streams_than_queues(tmp_path, monkeypatch):
    import bench
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")
    with pytest.raises(SystemExit, match="GPU_MAX_HW_QUEUES=8"):
        bench.run(bench.parse_args(["--streams", "8"]), 2, 0, 0, True)


def test_bench_world2_bad_gather_fails_the_shard_check(tmp_path):
    codes, logs, _ = _run_world(tmp_path, ["--gpus", "2"] + FAST, corrupt=True)
    assert codes == [3, 3]
    assert all("different shard" in lg["assertion"] for lg in logs)


# ---- ShardedFitness through the torch-free comm interface -----------------------------
def _sharded_rank(rank, world, mesh, B, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world), GGS_RDZV_DIR=out_dir, GGS_RDZV_KEY=f"sf-{B}")
    sys.path[:0] = [PKG, ORACLE]
    import _fakes
    import ggs_oracle as O
    from ggs.parallel import ShardedFitness, shard_bounds
    H, W = 32, 40
    pop = O.synthetic_population(B, 6, H, W, seed=5)
    tgt = np.random.default_rng(2).uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = np.random.default_rng(3).uniform(0.4, 1, (H, W)).astype(np.float32)
    seen = []

    def evaluate(G):
        seen.append(len(G))
        return O.fitness_many(list(G), tgt, H, W, 3.0, weight_mask=mask).astype(np.float32)

    comm = _fakes.PipeComm(mesh, rank, world)
    fit = ShardedFitness(tgt, H, W, weight_mask=mask, evaluate=evaluate, comm=comm)(pop)
    b0, b1 = shard_bounds(B, world, rank)
    ok = seen == ([b1 - b0] if b1 > b0 else [])
    np.save(os.path.join(out_dir, f"fit{rank}.npy"), fit)
    os._exit(0 if ok else 4)


@pytest.mark.parametrize("B,world", [(7, 2), (8, 2), (1, 2), (10, 3)])
def test_sharded_fitness_torch_free_world_n(tmp_path, B, world):
    import _fakes
    sys.path[:0] = [ORACLE]
    import ggs_oracle as O
    ctx = mp.get_context("fork")
    mesh = _fakes.PipeMesh(world, ctx)
    procs = [ctx.Process(target=_sharded_rank, args=(r, world, mesh, B, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert [p.exitcode for p in procs] == [0] * world
    H, W = 32, 40
    pop = O.synthetic_population(B, 6, H, W, seed=5)
    tgt = np.random.default_rng(2).uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = np.random.default_rng(3).uniform(0.4, 1, (H, W)).astype(np.float32)
    ref = O.fitness_many(list(pop), tgt, H, W, 3.0, weight_mask=mask).astype(np.float32)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"fit{r}.npy"), ref)


def test_rendezvous_ignores_an_id_left_by_an_earlier_launch(tmp_path, monkeypatch):
    """A crashed launch can leave its id file behind; a later launch with the same
    key must wait for rank 0's new file rather than read the stale one."""
    import time
    from ggs import parallel as P
    monkeypatch.setattr(P, "_RDZV_SEQ", [0])
    path = tmp_path / "ggs-rdzv-k-0-w2.id"
    path.write_bytes(b"\x01" * 128)
    old = time.time() - 3600
    os.utime(path, (old, old))
    monkeypatch.setattr(P, "launch_time", lambda: time.time() - 60)
    with pytest.raises(TimeoutError):
        P.file_rendezvous(1, 2, None, key="k", timeout_s=0.3, directory=str(tmp_path))
    monkeypatch.setattr(P, "_RDZV_SEQ", [0])
    path.write_bytes(b"\x02" * 128)                     # rank 0 of this launch
    assert P.file_rendezvous(1, 2, None, key="k", timeout_s=5, directory=str(tmp_path)) == b"\x02" * 128


def test_rccl_gather_refuses_a_multi_node_world(monkeypatch):
    """The file rendezvous is node-local: a WORLD_SIZE larger than this node's
    ranks fails at once instead of timing out (pass a torch group instead)."""
    from ggs import parallel as P
    monkeypatch.setenv("WORLD_SIZE", "16")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "9")
    monkeypatch.setattr(P, "_torch_dist_initialized", lambda: False)
    with pytest.raises(RuntimeError, match="LOCAL_WORLD_SIZE"):
        P.RcclGather(0)
