"""GA layer throughput: generations/s of ggs.ga.genetic_approx.

Presets (--preset):
  bench    512x512, 256 splats, pop 128, elite 8 (the BASELINE bench workload; default)
  default  the reference's shipped run (run_ggs.py:41 with modules/config.py:5-11):
           WORK_MAX_SIDE 512, N_SPLATS 512, POP_SIZE 32, ELITE_K 8, TOUR_K 2,
           CXPB 0.05, MUTPB 0.05 -> 24 offspring evaluated per generation
Explicit --size / --splats / --pop / --elite override the preset.

--backend host: host-side batched operators + one libggs launch per generation.
--backend device: the device-resident loop (ggs/ga_device.py), whole generations
on the GPU (Philox draws), timed around DeviceGA.run + a final read; then a second
run with libggs's HIP-event profiling on gives the per-generation device time of
breed / raster / finalize (events add host work, so that run is not the rate).

usage: python tools/bench_ga.py [--preset bench|default] [--gens 200] [--backend host|device]
       python -m torch.distributed.run --nproc-per-node G tools/bench_ga.py --backend device ...
           (configs[3]: --size 1024 --splats 1024 --pop 4096; offspring sharded over G GPUs)"""
import argparse, json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "genetic-gaussian-splats_amd"))
import ggs
from ggs import ga

PRESETS = {"bench": dict(size=512, splats=256, pop=128, elite=8),
           "default": dict(size=512, splats=512, pop=32, elite=8)}

ap = argparse.ArgumentParser()
ap.add_argument("--preset", default="bench", choices=sorted(PRESETS))
ap.add_argument("--gens", type=int, default=200)
ap.add_argument("--pop", type=int, default=0)
ap.add_argument("--splats", type=int, default=0)
ap.add_argument("--size", type=int, default=0)
ap.add_argument("--elite", type=int, default=-1)
ap.add_argument("--backend", default="host", choices=["host", "device"])
ap.add_argument("--profile-gens", type=int, default=200,
                help="device backend: generations of the HIP-event profiled run (0: skip)")
a = ap.parse_args()
pre = PRESETS[a.preset]
a.size = a.size or pre["size"]
a.splats = a.splats or pre["splats"]
a.pop = a.pop or pre["pop"]
a.elite = pre["elite"] if a.elite < 0 else a.elite
H = W = a.size
target = np.random.default_rng(0).uniform(0, 255, (H, W, 3)).astype(np.float32)
cfg = dict(mut_sigma_max={"xy": 0.1, "alog": 0.5, "blog": 0.5, "theta": 0.3, "rgb": 25.0, "alpha": 25.0},
           mut_sigma_min={"xy": 0.01, "alog": 0.05, "blog": 0.05, "theta": 0.025, "rgb": 2.0, "alpha": 2.0},
           schedule="cosine")
t_eval = [0.0]
from ggs.mask import compute_importance_mask, prepare_target
t = prepare_target(target, H, W)
m = compute_importance_mask(t, H, W, smooth=3, strength=0.7)
evaluated = a.pop - max(a.elite, 1)            # offspring[:P - E] survive (algorithm.py:140-141)
config = {"preset": a.preset, "H": H, "W": W, "splats": a.splats, "pop": a.pop, "elite": a.elite,
          "gens": a.gens, "evaluated_per_gen": evaluated}

if a.backend == "device":
    # under torch.distributed.run: one process per GPU, every rank runs the same
    # session and evaluates its shard of the offspring; one RCCL all-gather of the
    # fitness scalars per generation (ggs_ga_set_comm)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 or "TORCHELASTIC_RUN_ID" in os.environ:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from ggs.ga_device import DeviceGA
    init = ga.new_population(a.pop, a.splats, H, W, 3.0, 0.1, np.random.default_rng(0))
    dga = DeviceGA(t, m, init, tour_k=2, elite_k=a.elite, cxpb=0.05, mutpb=0.05, min_scale_splats=3.0,
                   max_scale_splats=0.1, seed=1, device=local, **cfg)
    gather = None
    if dist is not None:
        gather = ggs.RcclGather(local)
        dga.set_comm(gather)
    dga.run(1, 5, a.gens)                                          # warm-up
    dga.read()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    dga.run(6, a.gens, a.gens + 5)
    st = dga.read()
    dt = time.perf_counter() - t0
    if dist is not None:                                           # max over ranks; same GA everywhere
        out = [None] * world
        dist.all_gather_object(out, (dt, st["best_fit"], float(st["fitness"].sum())))
        dt = max(o[0] for o in out)
        assert len({o[1:] for o in out}) == 1, f"ranks diverged: {out}"
    kern = None
    if a.profile_gens > 0:                                         # per-generation device time
        ggs.profile_reset()
        ggs.profile_enable(True)
        g0 = a.gens + 6
        dga.run(g0, a.profile_gens, g0 + a.profile_gens)
        dga.read()
        ggs.profile_enable(False)
        kern = {}
        for name, k in (("breed", "prep"), ("raster", "raster"), ("finalize", "finalize")):
            ms, n = ggs.profile_read(k)
            kern[name + "_us"] = round(ms * 1e3 / max(n, 1), 2)
        kern["launches"] = {"raster": ggs.profile_read("raster")[1]}
    if rank == 0:
        print(json.dumps({"metric": "GA generations/s (device-resident)", "value": round(a.gens / dt, 2),
                          "config": dict(config, n_gpus=world, sharded=dist is not None),
                          "ms_per_gen": round(dt / a.gens * 1e3, 4),
                          # candidates rendered per generation: the P - elite_k surviving
                          # offspring (the reference renders all P offspring + the elites again)
                          "candidate_renders_per_s": round(a.gens * evaluated / dt, 1),
                          "reference_renders_per_gen": a.pop + a.elite,
                          "device_us_per_gen": kern,
                          "best_fit": st["best_fit"]}))
    dga.close()
    if gather is not None:
        gather.close()
    if dist is not None:
        dist.destroy_process_group()
    sys.exit(0)


def evaluate(G):
    t0 = time.perf_counter()
    f = ggs.fitness(G, t, H, W, 3.0, weight_mask=m)
    t_eval[0] += time.perf_counter() - t0
    return f

ga.genetic_approx(target, H, W, "cuda", a.pop, a.splats, 3, 2, a.elite, 0.05, 0.05, min_scale_splats=3.0,
                  max_scale_splats=0.1, k_sigma=3.0, mask_strength=0.7, boost_only=False, seed=0,
                  evaluate=evaluate, progress=False, **cfg)          # warm-up
t_eval[0] = 0.0
t0 = time.perf_counter()
best, fit = ga.genetic_approx(target, H, W, "cuda", a.pop, a.splats, a.gens, 2, a.elite, 0.05, 0.05,
                              min_scale_splats=3.0, max_scale_splats=0.1, k_sigma=3.0,
                              mask_strength=0.7, boost_only=False, seed=1, evaluate=evaluate,
                              progress=False, **cfg)
dt = time.perf_counter() - t0
print(json.dumps({"metric": "GA generations/s", "value": round(a.gens / dt, 2), "config": config,
                  "ms_per_gen": round(dt / a.gens * 1e3, 3),
                  "eval_ms_per_gen (host API incl. copies)": round(t_eval[0] / a.gens * 1e3, 3),
                  "host_ops_ms_per_gen": round((dt - t_eval[0]) / a.gens * 1e3, 3),
                  "best_fit": fit}))
