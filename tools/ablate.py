"""Time the raster kernel of several libggs builds on the bench workload.

usage: python tools/ablate.py lib1.so lib2.so ...   (each timed in its own
subprocess, interleaved rounds; prints median raster ms per build)."""
import json, os, subprocess, sys

CHILD = r'''
import os, sys, json, numpy as np, torch
sys.path.insert(0, "genetic-gaussian-splats_amd")
import bench, ggs
H = W = 512; N = 256; B = int(os.environ.get("ABL_B", "128"))
dev = torch.device("cuda", 0)
pops = [torch.from_numpy(bench.synthetic_population(B, N, i)).to(dev) for i in range(4)]
rng = np.random.default_rng(1234)
tgt = torch.from_numpy(rng.uniform(0, 1, (H, W, 3)).astype(np.float32)).to(dev)
mask = torch.from_numpy(rng.uniform(0.405, 1, (H, W)).astype(np.float32)).to(dev)
out = torch.empty(B, device=dev)
st = torch.cuda.current_stream(dev).cuda_stream
plan = ggs.TargetPlan(0, st, tgt.data_ptr(), mask.data_ptr(), 1, 1.0, H, W) if hasattr(ggs, "TargetPlan") else None
def step(i):
    if plan is not None:
        plan.fitness_device(st, pops[i % 4].data_ptr(), B, N, 9, 3.0, out.data_ptr())
    else:
        ggs.fitness_device(0, st, pops[i % 4].data_ptr(), B, N, 9, tgt.data_ptr(), mask.data_ptr(), 1, 1.0, H, W, 3.0, out.data_ptr())
for i in range(5): step(i)
torch.cuda.synchronize()
import time
t0 = time.perf_counter()
for i in range(40): step(i)
torch.cuda.synchronize()
step_ms = (time.perf_counter() - t0) / 40 * 1e3
ggs.profile_reset(); ggs.profile_enable(True)
for i in range(40): step(i)
torch.cuda.synchronize(); ggs.profile_enable(False)
ms, n = ggs.profile_read("raster")
print(json.dumps({"lib": os.environ["GGS_LIB"], "raster_ms": ms / n, "step_ms": step_ms}))
'''

libs = sys.argv[1:]
res = {l: [] for l in libs}
for rnd in range(3):
    for l in libs:
        env = dict(os.environ, GGS_LIB=os.path.abspath(l))
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print("FAILED", l, r.stderr[-2000:]); sys.exit(1)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        res[l].append((d["raster_ms"], d["step_ms"]))
for l, v in res.items():
    r = sorted(x[0] for x in v)
    st = sorted(x[1] for x in v)
    print(f"{os.path.basename(l):28s} raster median {r[len(r)//2]:.4f} ms (min {r[0]:.4f})   "
          f"step median {st[len(st)//2]:.4f} ms (min {st[0]:.4f})")
