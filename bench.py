#!/usr/bin/env python3
"""Benchmark of the reference's hot path on MI355X: candidate renders/s.

Workload (BASELINE.json `metric`, configs[1]): 512x512 canvas, 256 splats per
candidate, pop = 128 candidates per GPU, weighted-L2 fitness (the GA's default
path, fitness.py:28-31 with the importance mask) — one *step* = the evaluation
of one population of 128 candidates per GPU: encode + preprocess + raster + fused
weighted L2 + finalize (libggs.so, device-pointer API, inputs resident in HBM),
plus — for N > 1 GPUs — the RCCL all-gather of the fitness scalars (libggs
ggs_comm_allgather on the compute stream; the only exchange step; candidates
are sharded, weak scaling).  Consecutive populations are independent and
alternate over --streams HIP streams (default 4); `value_one_stream` is the rate
when each step must wait for the previous one (a GA generation).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--streams S] [--config 512|1024]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line.  Synthetic data: genomes drawn from the
population.py:20-46 distributions (4 different populations resident in HBM,
cycled step to step), target U[0,1], mask U[0.405,1].
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "genetic-gaussian-splats_amd"))

# BASELINE.json configs: [1] is the metric's workload (default); [2] is the
# 1024^2 / 1024-splat / pop-512 single-GPU case (--config 1024), whose per-GPU
# shard is also configs[3] (pop 4096 over 8 GPUs = 512 per GPU).
CONFIGS = {"512": (512, 256, 128), "1024": (1024, 1024, 512)}
H = W = 512
N_SPLATS = 256
POP = 128
K_SIGMA = 3.0
N_POPS = 4
RING = 8                         # in-flight fitness vectors (gather overlap)
# How the per-batch fitness all-gather is issued (A/B switch, tools/gather_exp.sh;
# "none" is a diagnostic, not a valid N>1 configuration):
#   "rccl"         (default) libggs's RCCL communicator, in order on the compute
#                  stream right after finalize: +1.5 us per step at world 1
#   "rccl-overlap" the same on the communicator's own stream, joined through the
#                  ring: +21 us (the cross-stream event waits cost more than they hide)
#   "torch" / "torch-sync"  torch.distributed all_gather_into_tensor, async through
#                  the ring / waited: +11 / +24 us
GATHER = os.environ.get("GGS_BENCH_GATHER", "rccl")
# Consecutive batches are independent populations, so they alternate over four
# HIP streams: one batch's raster fills the CUs the others' grid tails (and their
# prep/finalize launches) leave idle — tools/streams_exp.sh: 0.189 -> 0.173 ms
# per batch at two streams; four add 2 % more (tools/probe/streams_ab.sh,
# streams_tr.sh: 781-786k vs 766-768k renders/s, the same under torchrun;
# eight streams 763-768k, 16 hardware queues instead of 8 no different).
# A GA generation depends on the previous one's fitness and runs at the
# one-stream rate, reported beside as value_one_stream.
STREAMS = int(os.environ.get("GGS_BENCH_STREAMS", "4"))
# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default); under
# torchrun torch's and RCCL's streams take queues too and the second compute
# stream ends up sharing one (669k vs 730k renders/s at world 1), so ask for 8.
# Read by the HIP runtime at initialisation, which happens after this line.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
VALU_PEAK_TFLOPS = 157.3         # MI355X_MICROARCH.md: peak FP32 vector
FLOP_PER_PAIR = 24


def bytes_per_candidate():
    """algorithmic bytes per candidate, fused fitness = 12HW + 4HW + 36N + 4."""
    return 12 * H * W + 4 * H * W + 36 * N_SPLATS + 4


def synthetic_population(B, N, seed):
    """population.py:20-46 distributions (numpy RNG)."""
    rng = np.random.default_rng(seed)
    s_lo, s_hi = 3.0, 0.1 * max(H, W)

    def log_scales(m):
        u = rng.beta(m * 8 + 1e-6, (1 - m) * 8 + 1e-6, size=(B, N, 1))
        return np.log(s_lo + u * (s_hi - s_lo))

    G = np.concatenate([rng.uniform(0, 1, (B, N, 2)), log_scales(0.4), log_scales(0.6),
                        rng.uniform(-np.pi, np.pi, (B, N, 1)), rng.uniform(0, 256, (B, N, 3)),
                        rng.uniform(180, 256, (B, N, 1))], -1).astype(np.float32)
    G[..., 5:9] = np.clip(G[..., 5:9], 0, 255)
    return G


def _bench_profiles():
    """profiles/rNN/summary.json of this workload, oldest round first (the
    profiles/rNN_<config> directories hold the other configs)."""
    import glob
    import re
    return sorted(p for p in glob.glob(os.path.join(REPO, "profiles", "r*", "summary.json"))
                  if re.fullmatch(r"r\d+", os.path.basename(os.path.dirname(p))))


def pmc_traffic():
    """HBM bytes per raster launch from the newest committed rocprofv3 PMC
    summary of this same workload (tools/profile.sh -> profiles/rNN/summary.json:
    FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE); None when absent."""
    import glob
    paths = _bench_profiles()
    if not paths:
        return None, None
    try:
        d = json.load(open(paths[-1]))
        return d["raster_hbm_bytes_per_launch"]["total"], os.path.relpath(paths[-1], REPO)
    except (OSError, KeyError, ValueError):
        return None, None


def pmc_valu_busy():
    """Fraction of SIMD cycles the raster kernel's VALU was busy, from the same
    committed PMC summary: SQ_ACTIVE_INST_VALU (quad-cycles, summed over SIMDs)
    x 4 / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); None when absent."""
    import glob
    paths = _bench_profiles()
    if not paths:
        return None
    try:
        cs = json.load(open(paths[-1]))["counters"]
        c = cs[next(k for k in cs if "raster_kernel<1" in k)]
        return round(c["SQ_ACTIVE_INST_VALU"] * 4 / (c["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
    except (OSError, KeyError, ValueError, ZeroDivisionError, StopIteration):
        return None


def _cpu_worker(args):
    pop, tgt, mask = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import ggs_oracle as O
    return O.fitness_many(list(pop), tgt, H, W, K_SIGMA, weight_mask=mask)


def cpu_baseline(tgt, mask, per_worker=80):
    """The oracle (numpy restatement of render.py + fitness.py) timed on the
    host cores, candidates split over a process pool (80 per process: a ~10 s
    bounded sample of the same workload).  Runs BEFORE any GPU initialisation
    (fork)."""
    import multiprocessing as mp
    cores = max(1, min(16, os.cpu_count() or 1))
    pops = [synthetic_population(per_worker, N_SPLATS, 1000 + i) for i in range(cores)]
    ctx = mp.get_context("fork")
    with ctx.Pool(cores) as pool:
        pool.map(_cpu_worker, [(p[:1], tgt, mask) for p in pops])     # warm the workers
        t0 = time.perf_counter()
        pool.map(_cpu_worker, [(p, tgt, mask) for p in pops])
        dt = time.perf_counter() - t0
    n = cores * per_worker
    t1 = time.perf_counter()                                      # 1 core
    _cpu_worker((pops[0][:8], tgt, mask))
    one = 8 / (time.perf_counter() - t1)
    return {"value": n / dt, "unit": "candidate renders/s", "cores": cores, "kind": "port",
            "sample": f"{n} candidates ({per_worker} per process x {cores} processes, 1 thread each) "
                      f"at 512x512/256 splats, weighted fitness, oracle/ggs_oracle.py numpy; {dt:.1f} s",
            "single_core_value": round(one, 2), "cpu_model": _cpu_model(),
            "host_cpus_visible": os.cpu_count()}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="512")
    ap.add_argument("--ramp-ms", type=float, default=300.0,
                    help="untimed steps before the warm-up, until the clocks have ramped")
    ap.add_argument("--streams", type=int, default=STREAMS,
                    help="HIP streams the independent batches alternate over (1 = dependent batches)")
    ap.add_argument("--pop", type=int, default=0,
                    help="candidates per GPU per batch (0: the config's; other values explore batch size "
                         "and are not the BASELINE workload)")
    args = ap.parse_args()
    global H, W, N_SPLATS, POP
    H, N_SPLATS, POP = CONFIGS[args.config]
    W = H
    if args.pop > 0:
        POP = args.pop

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    rng = np.random.default_rng(1234)
    tgt_h = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask_h = rng.uniform(0.405, 1.0, (H, W)).astype(np.float32)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "512":
        cpu = cpu_baseline(tgt_h, mask_h)

    import torch
    import torch.distributed as dist
    import ggs

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ   # torchrun, even at N=1
    if distributed:
        dist.init_process_group("nccl", device_id=dev)

    pops = [torch.from_numpy(synthetic_population(POP, N_SPLATS, 10_000 * rank + i)).to(dev)
            for i in range(N_POPS)]
    tgt = torch.from_numpy(tgt_h).to(dev)
    mask = torch.from_numpy(mask_h).to(dev)
    # fitness vectors in a ring of slots: with an overlapped gather (A/B modes
    # below) batch i's gather reads outs[i % RING] while batch i+1 is evaluated
    # into the next slot; a slot is reused only after its gather (device-side wait)
    outs = [torch.empty(POP, dtype=torch.float32, device=dev) for _ in range(RING)]
    gathered = [torch.empty(POP * world, dtype=torch.float32, device=dev) for _ in range(RING)]
    works = [None] * RING
    stream = torch.cuda.current_stream(dev)
    st = stream.cuda_stream
    # batches alternate over STREAMS HIP streams (independent batches: the next
    # batch's raster fills the CUs the previous one's grid tail leaves idle)
    assert RING % args.streams == 0, f"--streams must divide {RING}"
    assert args.streams == 1 or not (distributed and GATHER.startswith("torch")), \
        "torch.distributed gathers run on torch's current stream: use --streams 1"
    sts = [st] + [torch.cuda.Stream(dev).cuda_stream for _ in range(args.streams - 1)]

    # the target/mask are fixed over a GA run: lay them out once for the raster's
    # fitness epilogue (ggs_plan_create), as the device-resident GA does
    plan = ggs.TargetPlan(local_rank, st, tgt.data_ptr(), mask.data_ptr(), ggs.GGS_FIT_WEIGHTED, 1.0,
                          H, W)

    # one RCCL communicator per stream: a communicator orders its collectives
    # across streams, which would serialise the alternating batches again
    comms = [ggs.RcclGather(local_rank) for _ in range(args.streams)] \
        if distributed and GATHER.startswith("rccl") else None
    comm = comms[0] if comms else None

    def join(j):                                             # slot j's stream waits for its gather
        if works[j] is None:
            return
        if comm is not None:
            k, ticket = works[j]                             # (stream/communicator index, ticket)
            comms[k].wait(sts[k], ticket)
        else:
            works[j].wait()
        works[j] = None

    def step(i, ns, gather=True):
        g, j, st = pops[i % N_POPS], i % RING, sts[i % ns]
        join(j)
        plan.fitness_device(st, g.data_ptr(), POP, N_SPLATS, 9, K_SIGMA, outs[j].data_ptr())
        if not distributed or GATHER == "none" or not gather:
            return
        if comm is not None:                                 # RCCL: fitness scalars to every rank
            works[j] = (i % ns, comms[i % ns].allgather(st, outs[j].data_ptr(), gathered[j].data_ptr(), POP,
                                                        overlap=GATHER == "rccl-overlap"))
        else:
            works[j] = dist.all_gather_into_tensor(gathered[j], outs[j], async_op=True)
        if GATHER == "torch-sync":
            join(j)

    def barrier():
        for j in range(RING):
            join(j)
        if distributed:
            dist.barrier()
        torch.cuda.synchronize(dev)

    # Clock ramp before any measurement: the GPU raises its clocks over tens of ms
    # of load (a 30-step run right after set-up measured the raster at 0.187-0.195
    # ms vs 0.178 ms in steady state), so run the evaluation untimed for --ramp-ms
    # first (no gathers: ranks may run different numbers of these steps).
    def ramp(ms, ns):
        t_ramp, i = time.perf_counter(), 0
        while (time.perf_counter() - t_ramp) * 1e3 < ms:
            for _ in range(50):
                step(i, ns, gather=False)
                i += 1
            torch.cuda.synchronize(dev)
        barrier()

    barrier()                  # first collective's one-time set-up before the ramp, not after it
    ramp(args.ramp_ms, args.streams)

    def timed(ns):
        """W untimed + K timed steps over ns streams, bracketed by barrier + synchronize:
        (this rank's seconds, host enqueue seconds); the max over ranks is taken
        once every pass has run."""
        for i in range(args.warmup):
            step(i, ns)
        barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(i, ns)
        host_s = time.perf_counter() - t0                   # enqueue time (host side)
        barrier()
        return time.perf_counter() - t0, host_s

    elapsed, host_s = timed(args.streams)                  # the headline
    if distributed and GATHER != "none":                    # the gather delivered this rank's shard
        j = (args.steps - 1) % RING
        shard_ok = torch.equal(gathered[j][rank * POP:(rank + 1) * POP], outs[j])
    # dependent batches (a GA generation needs the previous one's fitness): one stream
    # (each later pass gets a short ramp too: under torchrun the first passes after
    # a switch measured 5-15 % slow, tools/probe/pass_speed.py)
    if args.streams > 1:
        ramp(args.ramp_ms / 3, 1)
        elapsed1, _ = timed(1)
    else:
        elapsed1 = elapsed
    ramp(args.ramp_ms / 3, 1)

    # per-kernel device time (HIP events on the launch stream) over a third,
    # single-stream pass (kernels alone, not sharing the chip with the other
    # stream's): the raster kernel is the dominant one
    for rep in range(int(os.environ.get("GGS_BENCH_PROFILE_REPS", "1"))):
        ggs.profile_reset()
        ggs.profile_enable(True)
        for i in range(args.steps):
            step(i, 1)
        barrier()
        ggs.profile_enable(False)
        if os.environ.get("GGS_BENCH_PROFILE_REPS") and rank == 0:
            ms_, n_ = ggs.profile_read("raster")
            print(f"profile pass {rep}: raster {ms_ / max(n_, 1):.4f} ms", file=sys.stderr, flush=True)
    kern = {k: ggs.profile_read(k) for k in ("prep", "raster", "finalize")}
    raster_ms = kern["raster"][0] / max(kern["raster"][1], 1)
    # max over ranks, after every measured pass (a first all-reduce between the
    # passes idles the GPU long enough for the clocks to drop)
    if distributed:
        t = torch.tensor([elapsed, elapsed1], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, elapsed1 = (float(v) for v in t.tolist())
        if GATHER != "none":
            assert shard_ok, "fitness all-gather returned a different shard"

    # algorithmic work of this workload (AABB pairs from the product's own prep)
    pairs = 0
    for p in pops:
        pre = ggs.preprocess(ggs.encode(p.cpu().numpy()), H, W, K_SIGMA)
        pairs += int(((pre["x1"].astype(np.int64) - pre["x0"] + 1) *
                      (pre["y1"].astype(np.int64) - pre["y0"] + 1)).sum())
    pairs_per_cand = pairs / (N_POPS * POP)

    # PCIe-inclusive rate of the host API (numpy genomes in, fitness scalars out:
    # target/mask content check, pinned staging, 3 launches, D2H) — the path a
    # caller handing over host buffers gets; reported beside, never the value
    host_api = None
    if world == 1 and not distributed:
        hpops = [p.cpu().numpy() for p in pops]
        ggs.fitness(hpops[0], tgt_h, H, W, K_SIGMA, weight_mask=mask_h)
        n_h, t_h = 0, time.perf_counter()
        while time.perf_counter() - t_h < 0.5:
            ggs.fitness(hpops[n_h % N_POPS], tgt_h, H, W, K_SIGMA, weight_mask=mask_h)
            n_h += 1
        host_api = round(n_h * POP / (time.perf_counter() - t_h), 1)

    total = world * POP * args.steps
    value = total / elapsed
    raster_bytes = bytes_per_candidate() * POP
    achieved_gbs = raster_bytes / (raster_ms * 1e-3) / 1e9
    valu_tflops = FLOP_PER_PAIR * pairs_per_cand * POP / (raster_ms * 1e-3) / 1e12
    traffic, traffic_src = pmc_traffic() if args.config == "512" and POP == 128 else (None, None)
    if rank == 0:
        line = {
            "metric": "candidate renders/sec (and Gsplat-pixels/s), 512x512, 256 splats, pop=128"
                      if args.config == "512" and POP == 128 else
                      f"candidate renders/sec, {H}x{W}, {N_SPLATS} splats, pop={POP} per GPU",
            "value": round(value, 1),
            "unit": "candidate renders/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (population.py distributions, U[0,1] target, U[0.405,1] mask)",
            "config": {"workload": f"{H}x{W} canvas, {N_SPLATS} splats/candidate, pop={POP} per GPU, "
                                   "weighted-L2 fitness (encode+prep+raster+reduce)",
                       "H": H, "W": W, "splats": N_SPLATS, "pop_per_gpu": POP,
                       "global_batch": POP * world, "parallelism": f"dp{world} (candidate shards)",
                       "fitness_gather": (GATHER if distributed else None)},
            "gsplat_pixels_per_s": round(value * N_SPLATS * H * W / 1e9, 2),
            "aabb_pairs_per_s": round(value * pairs_per_cand, 1),
            "roofline": {"bound": "hbm", "kernel": "raster_kernel<1, false>",
                         "achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 5),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": raster_bytes,
                         "avg_launch_ms": round(raster_ms, 5),
                         "note": "VALU/transcendental-bound path (SURVEY.md §8d): see 'valu'"},
            "valu": {"achieved": round(valu_tflops, 3), "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(valu_tflops / VALU_PEAK_TFLOPS, 4),
                     "flop_per_aabb_pair": FLOP_PER_PAIR, "aabb_pairs_per_candidate": pairs_per_cand,
                     "accounting": "reference-equivalent work: 24 FLOP per AABB pair (SURVEY.md §8d); "
                                   "the row recurrence executes fewer, so frac can exceed 1",
                     "busy_pmc": pmc_valu_busy() if args.config == "512" and POP == 128 else None},
            "streams": args.streams,
            "value_one_stream": round(world * POP * args.steps / elapsed1, 1),
            "host_enqueue_ms_per_step": round(host_s / args.steps * 1e3, 4),
            "host_api_renders_per_s": host_api,
            "kernels_ms_per_launch": {k: round(v[0] / max(v[1], 1), 5) for k, v in kern.items()},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    for c in comms or ():
        c.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
