import os, sys, subprocess, json
code = r'''
import sys, hashlib, numpy as np
sys.path.insert(0, "genetic-gaussian-splats_amd"); sys.path.insert(0, "oracle")
import ggs, ggs_oracle as O
outs = []
for (H, W, B, N, s) in [(512, 512, 32, 256, 1), (250, 120, 3, 1100, 2), (64, 80, 5, 30, 3)]:
    pop = O.synthetic_population(B, N, H, W, seed=s)
    rng = np.random.default_rng(s)
    tgt = rng.uniform(0, 1, (H, W, 3)).astype(np.float32); m = rng.uniform(0.4, 1, (H, W)).astype(np.float32)
    for mask, boost in ((m, False), (None, False), (m, True)):
        outs.append(ggs.fitness(pop, tgt, H, W, 3.0, weight_mask=mask, boost_only=boost).tobytes().hex())
    outs.append(hashlib.sha1(ggs.render(ggs.encode(pop[:2]), H, W).tobytes()).hexdigest())
# thin, rotated, faint splats: the recurrence's seed guard trips on their far corners
rng = np.random.default_rng(7)
thin = O.synthetic_population(4, 200, 256, 256, seed=9)
thin[..., 2] = np.log(rng.uniform(40, 120, thin.shape[:2]))
thin[..., 3] = np.log(rng.uniform(1.0, 2.0, thin.shape[:2]))
thin[..., 8] = rng.uniform(0, 40, thin.shape[:2])
tgt = rng.uniform(0, 1, (256, 256, 3)).astype(np.float32)
outs.append(ggs.fitness(thin, tgt, 256, 256, 3.0).tobytes().hex())
outs.append(hashlib.sha1(ggs.render(ggs.encode(thin), 256, 256).tobytes()).hexdigest())
print("\n".join(outs))
'''
res = []
for lib in sys.argv[1:]:
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, GGS_LIB=os.path.abspath(lib)),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    res.append(r.stdout)
print("bit-identical" if all(x == res[0] for x in res) else "DIFFERENT")
