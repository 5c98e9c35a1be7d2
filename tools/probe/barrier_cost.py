"""Host time of the barrier variants bench.py could bracket its timed region with
(under torch.distributed.run, world 1 here)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "genetic-gaussian-splats_amd"))
import torch
import torch.distributed as dist
import ggs
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", device_id=dev)
t = torch.zeros(1, device=dev)
comm = ggs.RcclGather(0)
st = torch.cuda.current_stream(dev).cuda_stream
r = torch.zeros(dist.get_world_size(), device=dev)


def b_barrier():
    dist.barrier(); torch.cuda.synchronize(dev)


def b_allreduce():
    dist.all_reduce(t); torch.cuda.synchronize(dev)


def b_rccl():
    comm.allgather(st, t.data_ptr(), r.data_ptr(), 1); torch.cuda.synchronize(dev)


for name, fn in (("dist.barrier", b_barrier), ("all_reduce", b_allreduce), ("ggs rccl", b_rccl)):
    for _ in range(3):
        fn()
    t0 = time.perf_counter()
    for _ in range(20):
        fn()
    print(f"{name:14s} {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms", flush=True)
