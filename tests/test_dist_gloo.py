"""The multi-rank path (ggs.parallel) on CPU: world_size 2 over gloo, the
oracle injected as the per-rank evaluator.  Checks contiguous sharding, the
all-gather reassembly (ragged B), and equality with a single-process run."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ORACLE, PKG


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, B, out_path):
    import sys
    sys.path[:0] = [PKG, ORACLE]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
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

        fit = ShardedFitness(tgt, H, W, weight_mask=mask, evaluate=evaluate)(pop)
        b0, b1 = shard_bounds(B, world, rank)
        assert seen == ([b1 - b0] if b1 > b0 else [])
        np.save(f"{out_path}.{rank}.npy", fit)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B", [7, 8, 1])
def test_sharded_fitness_gloo_world2(tmp_path, B):
    import sys
    sys.path[:0] = [ORACLE]
    import ggs_oracle as O
    out = str(tmp_path / "fit")
    mp.start_processes(_worker, args=(2, _free_port(), B, out), nprocs=2, join=True,
                       start_method="spawn")
    H, W = 32, 40
    pop = O.synthetic_population(B, 6, H, W, seed=5)
    tgt = np.random.default_rng(2).uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask = np.random.default_rng(3).uniform(0.4, 1, (H, W)).astype(np.float32)
    ref = O.fitness_many(list(pop), tgt, H, W, 3.0, weight_mask=mask).astype(np.float32)
    for r in range(2):
        np.testing.assert_array_equal(np.load(f"{out}.{r}.npy"), ref)


def test_shard_bounds_cover_and_balance():
    from ggs.parallel import shard_bounds
    for B in (0, 1, 5, 128, 4096, 4097):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(B, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            per = -(-B // world)
            # equal ceil(B/world) slots (one in-place all-gather), only the tail short
            assert all(s == per for s in sizes[:B // per if per else 0])
            assert all(0 <= s <= per for s in sizes)
            assert all(a[0] == min(B, r * per) for r, a in enumerate(spans))
