"""Raster duration per 30-step pass over time, inside one process (plain or
under torch.distributed.run): does anything in the torchrun set-up slow the
kernels, and does it wear off?"""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "genetic-gaussian-splats_amd"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import torch
import bench, ggs
dist = None
if "TORCHELASTIC_RUN_ID" in os.environ:
    import torch.distributed as dist
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
dev = torch.device("cuda", 0)
H = W = 512
pops = [torch.from_numpy(bench.synthetic_population(128, 256, i)).to(dev) for i in range(4)]
rng = np.random.default_rng(1234)
tgt = torch.from_numpy(rng.uniform(0, 1, (H, W, 3)).astype(np.float32)).to(dev)
mask = torch.from_numpy(rng.uniform(0.405, 1, (H, W)).astype(np.float32)).to(dev)
out = torch.empty(128, device=dev)
gath = torch.empty(128, device=dev)
st = torch.cuda.current_stream(dev).cuda_stream
plan = ggs.TargetPlan(0, st, tgt.data_ptr(), mask.data_ptr(), 1, 1.0, H, W)
comm = ggs.RcclGather(0) if (dist is not None and os.environ.get("PS_COMM", "1") == "1") else None
t0 = time.perf_counter()
for p in range(12):
    if dist is not None and os.environ.get("PS_BARRIER", "1") == "1":
        dist.barrier()
    torch.cuda.synchronize()
    ggs.profile_reset(); ggs.profile_enable(True)
    for i in range(30):
        plan.fitness_device(st, pops[i % 4].data_ptr(), 128, 256, 9, 3.0, out.data_ptr())
        if comm is not None and os.environ.get("PS_GATHER", "0") == "1":
            comm.allgather(st, out.data_ptr(), gath.data_ptr(), 128)
    torch.cuda.synchronize(); ggs.profile_enable(False)
    ms, n = ggs.profile_read("raster")
    print(f"pass {p:2d} t={time.perf_counter() - t0:6.2f}s raster {ms / n:.4f} ms", flush=True)
