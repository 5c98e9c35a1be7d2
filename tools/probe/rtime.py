"""A/B timing of libggs builds: raster ms per launch (HIP events on the launch
stream) and one-stream step ms (prep + raster + finalize, dependent batches) at a
bench config, each build in its own process, builds alternated for --rounds.

    python tools/probe/rtime.py [--config 512|1024|1024x8|sa16|sa4|sa2|sa1|ga24] [--same] [--rounds 3] lib1.so lib2.so,KEY=VAL ...

Prints one line per (round, lib) and a median summary, which compares every build's
fitness vector with the first's (bit-identical or the max relative diff).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CFG = {"512": (512, 256, 128), "1024": (1024, 1024, 512), "1024x8": (1024, 1024, 4096), "sa16": (2048, 4096, 16),
       "sa2": (2048, 4096, 2), "sa4": (2048, 4096, 4), "sa1": (2048, 4096, 1),    # sa1: a lone SA neighbour (start of a run)
       "ga24": (512, 512, 24)}   # ga24: the shipped GA run's launch (config.py)


def worker(cfg, steps, out_npy, same=False):
    sys.path[:0] = [REPO, os.path.join(REPO, "genetic-gaussian-splats_amd")]
    os.environ.setdefault("GGS_HIP_RUNTIME", "system")
    import bench
    import ggs
    from ggs import hip
    H, N, P = CFG[cfg]
    bench.H = bench.W = H
    ggs.ensure_init()
    hip.set_device(0)
    pops = [bench.synthetic_population(P, N, 10_000 + i) for i in range(4)]
    if same:                 # every candidate a copy of the first (SA neighbours ~ the state)
        pops = [np.ascontiguousarray(np.broadcast_to(pops[0][:1], pops[0].shape))] * 4
    pops = [hip.DeviceArray.from_host(p) for p in pops]
    rng = np.random.default_rng(1234)
    tgt = hip.DeviceArray.from_host(rng.uniform(0, 1, (H, H, 3)).astype(np.float32))
    mask = hip.DeviceArray.from_host(rng.uniform(0.405, 1.0, (H, H)).astype(np.float32))
    out = hip.DeviceArray((P,))
    st = hip.Stream()
    plan = ggs.TargetPlan(0, st.handle, tgt.ptr, mask.ptr, ggs.GGS_FIT_WEIGHTED, 1.0, H, H)

    def run(n):
        for i in range(n):
            plan.fitness_device(st.handle, pops[i % 4].ptr, P, N, 9, 3.0, out.ptr)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.4:          # clock ramp
        run(20)
        st.synchronize()
    st.synchronize()
    t0 = time.perf_counter()
    run(steps)
    st.synchronize()
    step_ms = (time.perf_counter() - t0) / steps * 1e3
    ggs.profile_reset()
    ggs.profile_enable(True)
    run(steps)
    st.synchronize()
    ggs.profile_enable(False)
    ms, n = ggs.profile_read("raster")
    plan.fitness_device(st.handle, pops[0].ptr, P, N, 9, 3.0, out.ptr)
    np.save(out_npy, out.to_host(st))
    print(json.dumps({"raster_ms": ms / n, "step_ms": step_ms}))


def label(lib):
    path, *kv = lib.split(",")
    return ",".join([os.path.basename(path)] + [os.path.basename(x) for x in kv])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--config", default="512", choices=sorted(CFG))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--out", default="")
    ap.add_argument("--same", action="store_true", help="candidates of a launch identical (SA-like)")
    a = ap.parse_args()
    steps = a.steps or {"512": 300, "1024": 20, "1024x8": 4, "sa16": 60, "sa2": 200, "sa4": 120, "sa1": 300, "ga24": 600}[a.config]
    if a.worker:
        worker(a.config, steps, a.out, a.same)
        return
    res = {lib: [] for lib in a.libs}
    fits = {}
    for r in range(a.rounds):
        for lib in a.libs:
            # a lib may carry extra environment: path.so,KEY=VAL,KEY2=VAL2
            path, *kv = lib.split(",")
            npy = f"/tmp/rtime_{abs(hash(lib))}.npy"
            env = dict(os.environ, GGS_LIB=os.path.abspath(path), **dict(x.split("=", 1) for x in kv))
            p = subprocess.run([sys.executable, __file__, "--worker", "--config", a.config, "--steps", str(steps),
                                "--out", npy] + (["--same"] if a.same else []), env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-3000:])
                sys.exit(p.returncode)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            res[lib].append(d)
            fits[lib] = np.load(npy)
            print(f"round {r} {label(lib):28s} raster {d['raster_ms']:.5f} ms  step {d['step_ms']:.5f} ms",
                  flush=True)
    base = a.libs[0]
    for lib in a.libs:
        rm = np.median([d["raster_ms"] for d in res[lib]])
        sm = np.median([d["step_ms"] for d in res[lib]])
        f0, f1 = fits[base], fits[lib]
        same = "bit-identical" if np.array_equal(f0, f1) else f"max rel {np.max(np.abs(f1 - f0) / np.abs(f0)):.2e}"
        print(f"SUMMARY {a.config} {label(lib):28s} raster {rm:.5f} ms  step {sm:.5f} ms  "
              f"({(rm / np.median([d['raster_ms'] for d in res[base]]) - 1) * 100:+.2f}% raster)  {same}", flush=True)


if __name__ == "__main__":
    main()
