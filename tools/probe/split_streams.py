"""Dependent batches split over two HIP streams: does joining them with events
every step cost less than the grid tail it fills?

Step (a GA generation's evaluation, dependent on the previous step):
  1 stream : fitness(128 candidates) on stream A
  split    : A records e0; B waits e0; A: fitness(cands 0..63), B: fitness(64..127);
             A waits B's event (next step depends on both halves)
Prints ms per step for each (median of 3 rounds)."""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "genetic-gaussian-splats_amd"))
import torch
import bench
import ggs

H = W = 512
N, B = 256, 128
dev = torch.device("cuda", 0)
pops = [torch.from_numpy(bench.synthetic_population(B, N, i)).to(dev) for i in range(4)]
rng = np.random.default_rng(1234)
tgt = torch.from_numpy(rng.uniform(0, 1, (H, W, 3)).astype(np.float32)).to(dev)
mask = torch.from_numpy(rng.uniform(0.405, 1, (H, W)).astype(np.float32)).to(dev)
out = torch.empty(B, device=dev)
sA = torch.cuda.current_stream(dev)
sB = torch.cuda.Stream(dev)
plan = ggs.TargetPlan(0, sA.cuda_stream, tgt.data_ptr(), mask.data_ptr(), 1, 1.0, H, W)
half = B // 2
row = N * 9 * 4


def one(i):
    plan.fitness_device(sA.cuda_stream, pops[i % 4].data_ptr(), B, N, 9, 3.0, out.data_ptr())


def split(i, frac=0.5):
    k = int(B * frac)
    e0 = torch.cuda.Event()
    e0.record(sA)
    sB.wait_event(e0)
    g = pops[i % 4].data_ptr()
    plan.fitness_device(sA.cuda_stream, g, k, N, 9, 3.0, out.data_ptr())
    plan.fitness_device(sB.cuda_stream, g + k * row, B - k, N, 9, 3.0, out.data_ptr() + 4 * k)
    e1 = torch.cuda.Event()
    e1.record(sB)
    sA.wait_event(e1)


def timeit(fn, steps=300):
    for i in range(20):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fn(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


res = {}
for r in range(3):
    for name, fn in (("one_stream", one), ("split_50", split), ("split_75", lambda i: split(i, 0.75)),
                     ("split_85", lambda i: split(i, 0.85))):
        res.setdefault(name, []).append(timeit(fn))
for k, v in res.items():
    print(f"{k:12s} {sorted(v)[1]:.4f} ms/step")
