import os, sys, time, numpy as np
sys.path.insert(0, 'genetic-gaussian-splats_amd'); sys.path.insert(0, '.')
import bench, ggs
H=W=512; P=128
pop = bench.synthetic_population(P, 256, 1)
rng = np.random.default_rng(1234)
tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32); mask = rng.uniform(0.405, 1.0, (H, W)).astype(np.float32)
for _ in range(20): ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask)
t0=time.perf_counter(); n=0
while time.perf_counter()-t0 < 1.0:
    ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask); n+=1
dt=(time.perf_counter()-t0)/n
print(f"host API: {dt*1e6:.1f} us per call, {P/dt:.0f} renders/s")
dst=np.empty_like(pop)
t0=time.perf_counter()
for _ in range(200): np.copyto(dst, pop)
print(f"memcpy 1.18 MB: {(time.perf_counter()-t0)/200*1e6:.1f} us")
import xxhash
buf=np.concatenate([tgt.ravel(), mask.ravel()]).tobytes()
t0=time.perf_counter()
for _ in range(100): xxhash.xxh64(buf).intdigest()
print(f"xxh64 4 MB: {(time.perf_counter()-t0)/100*1e6:.1f} us")
