#!/usr/bin/env python3
"""Benchmark of the reference's hot path on MI355X: candidate renders/s.

Workload (BASELINE.json `metric`, configs[1]): 512x512 canvas, 256 splats per
candidate, pop = 128 candidates per GPU, weighted-L2 fitness (the GA's default
path, fitness.py:28-31 with the importance mask).  One *step* = the evaluation
of one population: encode + preprocess + raster + fused weighted L2 + finalize
(libggs.so, device-pointer API, inputs resident in HBM) and — on more than one
GPU — the RCCL all-gather of the fitness scalars (libggs ggs_comm_allgather on
the compute stream; the only exchange step).  Consecutive populations are
independent and alternate over --streams HIP streams (default 4);
`value_one_stream` is the rate when each step must wait for the previous one (a
GA generation), `value_with_readback` adds the per-step D2H of the B fitness
scalars (fitness.py:42 `.cpu()`).

No PyTorch anywhere (north_star): device memory and streams come from ggs.hip
(ctypes over the HIP runtime libggs uses), the collectives from libggs's own RCCL
communicators, their id from a file rendezvous on the node.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--streams S]
                    [--config 512|1024|1024x8]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

`--gpus N` outside a launcher starts N rank processes itself (before anything
touches a GPU) with RANK / LOCAL_RANK / WORLD_SIZE set, exactly what torchrun
would; under a launcher WORLD_SIZE must equal N.  Rank 0 prints ONE JSON line.

Configs: "512" (default; configs[1], weak scaling: 128 candidates per GPU),
"1024" (configs[2]: 1024^2 / 1024 splats / 512 per GPU, weak) and "1024x8"
(configs[3]: 1024^2 / 1024 splats, ONE population of 4096 split over the N GPUs,
strong scaling).  Synthetic data: genomes from the population.py:20-46
distributions (4 populations resident in HBM, cycled step to step), target
U[0,1], mask U[0.405,1].

Timing: W untimed steps, then passes of exactly K steps, each bracketed by a
barrier + device synchronize on both sides; passes repeat until >= --min-time
seconds were measured (the driver's --steps 20 is ~3 ms, inside launch/clock
jitter); the reported time is the median pass, after taking the max over ranks
pass by pass.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "genetic-gaussian-splats_amd"))

# name -> (H = W, splats, candidates, scaling).  "1024x8": the candidates are the
# GLOBAL population, split over the ranks (strong scaling); otherwise per GPU.
CONFIGS = {"512": (512, 256, 128, "weak"), "1024": (1024, 1024, 512, "weak"),
           "1024x8": (1024, 1024, 4096, "strong")}
H = W = 512
N_SPLATS = 256
POP = 128
K_SIGMA = 3.0
N_POPS = 4
RING = 8                         # in-flight fitness vectors (gather overlap)
METRIC = "candidate renders/sec (and Gsplat-pixels/s), 512x512, 256 splats, pop=128"
# How the per-step fitness all-gather is issued (A/B switch; docs/EXPERIMENTS.md §5):
#   "rccl"          (default) libggs's RCCL communicator, in order on the compute
#                   stream right after finalize: +1.5 us per step at world 1
#   "rccl-overlap"  the same on the communicator's own stream, joined through the
#                   ring: +21 us (the cross-stream event waits cost more than they hide)
#   "none"          diagnostic only, not a valid N > 1 configuration
GATHER = os.environ.get("GGS_BENCH_GATHER", "rccl")
# Consecutive batches are independent populations, so they alternate over four
# HIP streams: one batch's raster fills the CUs the others' grid tails (and their
# prep/finalize launches) leave idle (docs/EXPERIMENTS.md §5: 781-786k vs 766-768k
# renders/s at two streams, eight 763-768k).
STREAMS = int(os.environ.get("GGS_BENCH_STREAMS", "4"))
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


def _bench_profiles(config="512"):
    """profiles/rNN/summary.json of the headline workload (config "512"), or
    profiles/rNN_<config>/summary.json of another bench config, oldest round first."""
    import glob
    import re
    pat = r"r\d+" if config == "512" else r"r\d+_" + re.escape(config)
    return sorted(p for p in glob.glob(os.path.join(REPO, "profiles", "r*", "summary.json"))
                  if re.fullmatch(pat, os.path.basename(os.path.dirname(p))))


def _summary(config="512"):
    paths = _bench_profiles(config)
    if not paths:
        return None, None
    try:
        return json.load(open(paths[-1])), os.path.relpath(paths[-1], REPO)
    except (OSError, ValueError):
        return None, None


def _norm_kernel(k):
    return (k or "").replace("void ", "").replace("ggs::", "").strip()


def lib_sha256(path):
    import hashlib
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def profile_match(config, kernel, lib_sha):
    """Whether the newest committed profile of this launch shape describes THIS
    binary: its stamp (tools/prof_summary.py + tools/collect_profile.sh) must name
    exactly the raster instance this launch runs and the sha256 of the libggs.so
    this process loaded.  Returns (ok, reason, source)."""
    d, src = _summary(config)
    if d is None:
        return False, "no committed profile of this launch shape", None
    st = d.get("stamp") or {}
    prof_k = st.get("raster_kernel")
    if not prof_k:
        return False, f"{src} is not stamped with the profiled raster kernel and library", src
    if _norm_kernel(prof_k) != _norm_kernel(kernel):
        return False, f"{src} profiled {prof_k}; this launch runs {kernel}", src
    if st.get("libggs_sha256") != lib_sha:
        return False, (f"{src} profiled libggs.so sha256 {str(st.get('libggs_sha256'))[:16]}; this run loaded "
                       f"{str(lib_sha)[:16]}"), src
    return True, f"{src}: same raster instance, same libggs.so (git {str(st.get('git_head'))[:12]})", src


def _raster_counters(d):
    st = (d or {}).get("stamp") or {}
    k = st.get("raster_kernel")
    return d["counters"][k] if k else None


def pmc_traffic(config="512"):
    """HBM bytes per raster launch from the newest committed rocprofv3 PMC
    summary of this same workload (tools/profile.sh -> profiles/rNN[_<config>]/
    summary.json: FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE); None when absent."""
    d, src = _summary(config)
    try:
        return d["raster_hbm_bytes_per_launch"]["total"], src
    except (TypeError, KeyError):
        return None, None


def pmc_valu_busy(config="512"):
    """Fraction of SIMD cycles the raster kernel's VALU was busy, from the same
    committed PMC summary: SQ_ACTIVE_INST_VALU (quad-cycles, summed over SIMDs)
    x 4 / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) of the stamped raster kernel;
    None when absent."""
    d, _ = _summary(config)
    try:
        c = _raster_counters(d)
        return round(c["SQ_ACTIVE_INST_VALU"] * 4 / (c["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
    except (TypeError, KeyError, ZeroDivisionError):
        return None


def pmc_trace_avg_us(config="512"):
    """The committed rocprofv3 kernel-trace average of the raster kernel over a
    single-stream bench pass (tools/profile.sh runs bench.py --streams 1)."""
    d, _ = _summary(config)
    try:
        k = d["stamp"]["raster_kernel"]
        return d.get("raster_profile_pass_avg_us") or d["kernels"][k]["avg_us"]
    except (AttributeError, KeyError, TypeError):
        return None


def rocprof_kernel_ms(config="512"):
    """Per-kernel average durations (ms) of the committed rocprofv3 trace of this
    launch shape: prep, raster, finalize (the trace's own clock, beside the
    HIP-event figures, which include each event pair's overhead)."""
    d, _ = _summary(config)
    out = {}
    for name, key in (("prep", "prep_kernel<true>"), ("raster", None), ("finalize", "finalize_kernel")):
        try:
            k = d["stamp"]["raster_kernel"] if key is None else next(x for x in d["kernels"] if key in x)
            out[name] = round(d["kernels"][k]["avg_us"] / 1e3, 5)
        except (AttributeError, KeyError, TypeError, StopIteration):
            out[name] = None
    return out


def profile_config(config, pop_arg, per_gpu):
    """The bench config whose committed profile has this launch's shape: the config
    itself at its own batch; else the config launching the same (size, splats,
    candidates per GPU) — configs[3] split over 8 ranks is configs[2]'s launch;
    None for a --pop exploration nothing profiled."""
    Hc, Nc, Pc, _ = CONFIGS[config]
    if pop_arg <= 0 and per_gpu == Pc:
        return config
    return next((c for c, v in CONFIGS.items() if v[:3] == (Hc, Nc, per_gpu)), None)


# ---- CPU baseline -----------------------------------------------------------------
def _cpu_worker(args):
    pop, tgt, mask = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import ggs_oracle as O
    return O.fitness_many(list(pop), tgt, H, W, K_SIGMA, weight_mask=mask)


def cpu_cores():
    """The host cores this job may use: the CPU affinity set, capped by the
    box's per-job thread budget (OMP_NUM_THREADS; the GPU box grants 16 of its
    256 CPUs to a one-GPU job, so os.cpu_count() overstates what runs)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_baseline(tgt, mask, per_worker=80):
    """The oracle (numpy restatement of render.py + fitness.py) timed on the
    host cores, candidates split over a process pool (80 per process: a ~10 s
    bounded sample of the same workload).  Runs BEFORE any GPU initialisation
    (fork).  BASELINE.md's plan: 1 process, and one process per core."""
    import multiprocessing as mp
    cores = cpu_cores()
    pops = [synthetic_population(per_worker, N_SPLATS, 1000 + i) for i in range(cores)]
    ctx = mp.get_context("fork")
    with ctx.Pool(cores) as pool:
        pool.map(_cpu_worker, [(p[:1], tgt, mask) for p in pops])     # warm the workers
        t0 = time.perf_counter()
        pool.map(_cpu_worker, [(p, tgt, mask) for p in pops])
        dt = time.perf_counter() - t0
    n = cores * per_worker
    t1 = time.perf_counter()                                      # 1 core
    _cpu_worker((pops[0][:24], tgt, mask))
    one = 24 / (time.perf_counter() - t1)
    return {"value": round(n / dt, 2), "unit": "candidate renders/s", "cores": cores, "kind": "port",
            "sample": f"{n} candidates ({per_worker} per process x {cores} processes, 1 thread each) "
                      f"at {H}x{W}/{N_SPLATS} splats, weighted fitness, oracle/ggs_oracle.py numpy; "
                      f"{dt:.1f} s",
            "single_core_value": round(one, 2), "single_core_sample": "24 candidates, 1 process",
            "cpu_model": _cpu_model(), "host_cpus_visible": os.cpu_count(),
            "cores_rule": "CPU affinity set capped by OMP_NUM_THREADS (the job's CPU share on the "
                          "GPU box; os.cpu_count() counts the whole host)"}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ---- rank spawning (--gpus N outside a launcher) ----------------------------------
def visible_gpus():
    """GPUs this process could open, counted WITHOUT initialising HIP (the KFD
    topology: nodes with SIMDs), narrowed by the *_VISIBLE_DEVICES lists; None
    when unknown."""
    import glob
    n = 0
    try:
        for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
            for line in open(p):
                if line.startswith("simd_count") and int(line.split()[1]) > 0:
                    n += 1
    except (OSError, ValueError):
        return None
    if n == 0:
        return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv, python=sys.executable, script=None, gpus_visible=None) -> int:
    """Run this script as n rank processes (one per GPU) and return the job's
    exit code: the first failing rank's (the others are then stopped), else 0.
    The parent never touches a GPU: it only counts the KFD nodes."""
    have = visible_gpus() if gpus_visible is None else gpus_visible
    if have is not None and have < n:
        print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr, flush=True)
        return 2
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   GGS_RDZV_KEY=f"bench-{os.getpid()}-{port}")
        procs.append(subprocess.Popen([python, script or os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:                   # the job failed: stop the other ranks
                    q.terminate()
        time.sleep(0.05)
    return rc


# ---- hang watchdog (N > 1 must fail loudly, never hang) -----------------------------
WATCHDOG_EXIT = 124


def launch_key() -> str:
    """The key every rank of this launch shares (ggs.parallel.rendezvous_key)."""
    try:
        from ggs.parallel import rendezvous_key
        return rendezvous_key()
    except ImportError:
        return os.environ.get("GGS_RDZV_KEY") or f"run-{os.environ.get('MASTER_PORT', '0')}-{os.getppid()}"


class Watchdog:
    """A deadline on every phase of the run (communicator set-up, ramps, timed
    passes, the extra passes).  The main thread only stores where it is — phase,
    step, stream, and per communicator the collectives it has ISSUED (an in-stream
    RCCL gather is issued once its enqueue returned; a host collective once it was
    entered) — plain attribute stores, nothing on the hot path waits.  A daemon
    thread writes that state to a heartbeat file beside the RCCL id files every
    ``period`` s; when a phase outlives its deadline it reads every rank's
    heartbeat, names the rank(s) that issued the fewest collectives (the rank the
    others wait for), prints every rank's position to stderr and ends this process
    with WATCHDOG_EXIT.  No retry, no re-exec.  When no rank is behind, the hang is
    on the device (a kernel or a collective that never finishes) and the report
    says so."""

    def __init__(self, rank: int, world: int, key: str, directory=None, period: float = 0.5):
        import tempfile
        import threading
        self.rank, self.world, self.period = rank, world, period
        self.dir = directory or os.environ.get("GGS_RDZV_DIR") or tempfile.gettempdir()
        self.key = key
        self.phase, self.step, self.stream = "start", -1, -1
        self.issued = {}                              # communicator -> collectives issued
        self.last_ticket = None
        self.deadline = None
        self.budget = 0.0
        self.t_arm = time.monotonic()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="bench-watchdog", daemon=True)
        self._thread.start()

    def path(self, r: int) -> str:
        return os.path.join(self.dir, f"ggs-hb-{self.key}-r{r}.json")

    # ---- main thread -------------------------------------------------------------------
    def arm(self, phase: str, seconds: float) -> None:
        self.phase, self.budget, self.t_arm = phase, float(seconds), time.monotonic()
        self.deadline = self.t_arm + float(seconds)

    def disarm(self) -> None:
        self.deadline = None

    def collective(self, comm: int, ticket=None) -> None:
        self.issued[comm] = self.issued.get(comm, 0) + 1
        if ticket is not None:
            self.last_ticket = ticket

    def close(self) -> None:
        self._stop.set()
        self._thread.join(2 * self.period + 1)
        try:
            os.unlink(self.path(self.rank))
        except OSError:
            pass

    # ---- watchdog thread ---------------------------------------------------------------
    def state(self) -> dict:
        issued = dict(self.issued)          # one C-level copy: the main thread may add a key
        return {"rank": self.rank, "phase": self.phase, "step": self.step, "stream": self.stream,
                "issued": {str(k): v for k, v in sorted(issued.items())},
                "issued_total": sum(issued.values()), "last_ticket": self.last_ticket,
                "in_phase_s": round(time.monotonic() - self.t_arm, 3), "wall": time.time()}

    def _write(self) -> None:
        tmp = f"{self.path(self.rank)}.{os.getpid()}.tmp"
        try:
            with open(tmp, "w") as f:
                json.dump(self.state(), f)
            os.replace(tmp, self.path(self.rank))
        except OSError:
            pass

    def _run(self) -> None:
        while not self._stop.wait(self.period):
            try:
                self._write()
            except Exception:  # noqa: BLE001 — a heartbeat write never stops the watchdog
                pass
            d = self.deadline
            if d is not None and time.monotonic() > d:
                self._expire()

    def peers(self) -> dict:
        out = {}
        for r in range(self.world):
            try:
                with open(self.path(r)) as f:
                    out[r] = json.load(f)
            except (OSError, ValueError):
                out[r] = None
        return out

    @staticmethod
    def stalled(peers: dict, now: float, stale_s: float):
        """(ranks named as stalled, reason).  A rank whose heartbeat is missing or
        older than ``stale_s`` is frozen or gone; otherwise the ranks that issued
        the fewest collectives hold everyone else up; all equal: a device hang."""
        gone = [r for r, s in peers.items() if s is None or now - s["wall"] > stale_s]
        if gone:
            return gone, "no heartbeat (process frozen or gone)"
        counts = {r: s["issued_total"] for r, s in peers.items()}
        lo, hi = min(counts.values()), max(counts.values())
        if lo < hi:
            return sorted(r for r, c in counts.items() if c == lo), \
                f"issued {lo} collectives while the others issued up to {hi}"
        return [], f"every rank issued the same {lo} collectives: the hang is on the device"

    def _expire(self) -> None:
        self._write()
        time.sleep(min(self.period, 0.2))
        peers = self.peers()
        bad, why = self.stalled(peers, time.time(), stale_s=10 * self.period + 2)
        s = self.state()
        lines = [f"bench.py watchdog: rank {self.rank}: phase '{self.phase}' exceeded its "
                 f"{self.budget:.1f} s deadline (step {s['step']}, stream {s['stream']}, "
                 f"collectives issued per communicator {s['issued']}, last gather ticket "
                 f"{s['last_ticket']})",
                 f"bench.py watchdog: stalled rank(s): {bad if bad else 'none identified'} — {why}"]
        for r, p in sorted(peers.items()):
            lines.append(f"bench.py watchdog:   rank {r}: " + ("no heartbeat" if p is None else
                         f"phase '{p['phase']}' step {p['step']} stream {p['stream']} issued {p['issued']} "
                         f"last ticket {p['last_ticket']} ({p['in_phase_s']:.1f} s in phase)"))
        sys.stderr.write("\n".join(lines) + "\n")
        sys.stderr.flush()
        os._exit(WATCHDOG_EXIT)


def stream_accounting(n_streams: int, distributed: bool, gather: str, hw_queues: int) -> dict:
    """The HIP streams this process holds against GPU_MAX_HW_QUEUES.  Streams
    that carry collectives: the compute streams (in-stream gathers) or, with
    "rccl-overlap", each communicator's own stream; plus communicator 0's own
    stream, which runs the host-side barrier / max-over-ranks gathers.  RCCL's
    internal streams (about two per communicator) carry no gather kernel of ours.
    Two collective-carrying streams on one hardware queue would serialise one
    rank's gathers behind another's, so more of them than queues is refused."""
    comms = n_streams if distributed and gather.startswith("rccl") else 0
    own = 0 if not comms else (comms if gather == "rccl-overlap" else 1)
    carrying = 0 if not comms else (own if gather == "rccl-overlap" else n_streams + own)
    return {"compute_streams": n_streams, "communicators": comms, "communicator_streams": own,
            "rccl_internal_streams_est": 2 * comms, "total_est": n_streams + own + 2 * comms,
            "collective_streams": carrying, "gpu_max_hw_queues": hw_queues,
            "ok": carrying <= hw_queues}


# ---- the benchmark ---------------------------------------------------------------------
def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="512")
    ap.add_argument("--min-time", type=float, default=0.5,
                    help="repeat the K-step timed pass until this many seconds were measured")
    ap.add_argument("--ramp-ms", type=float, default=300.0,
                    help="untimed steps before the warm-up, until the clocks have ramped")
    ap.add_argument("--streams", type=int, default=STREAMS,
                    help="HIP streams the independent batches alternate over (1 = dependent batches)")
    ap.add_argument("--pop", type=int, default=0,
                    help="candidates per GPU per batch (0: the config's; other values explore batch size "
                         "and are not the BASELINE workload)")
    ap.add_argument("--extras", type=int, default=1,
                    help="0: headline pass only (profiling runs)")
    ap.add_argument("--watchdog-init-s", type=float, default=300.0,
                    help="deadline of the communicator set-up and the first barrier")
    ap.add_argument("--watchdog-floor-s", type=float, default=30.0,
                    help="every later phase's deadline: this floor + 20x its expected time from the "
                         "step time measured locally in the ramp")
    return ap.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:] if argv is None else argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ   # a launcher, even at N=1
    run(args, world, rank, local_rank, distributed)


def run(args, world, rank, local_rank, distributed):
    global H, W, N_SPLATS, POP
    # no torch in this process: /opt/rocm's HIP runtime and RCCL.  Set before anything
    # imports ggs (launch_key below does: the round-5 line ran on torch's runtime)
    os.environ.setdefault("GGS_HIP_RUNTIME", "system")
    H, N_SPLATS, pop_cfg, scaling = CONFIGS[args.config]
    W = H
    if scaling == "strong":                      # configs[3]: one population split over the ranks
        POP = -(-pop_cfg // world)
        global_batch = pop_cfg
    else:
        POP = args.pop if args.pop > 0 else pop_cfg
        global_batch = POP * world
    headline = args.config == "512" and POP == 128

    rng = np.random.default_rng(1234)
    tgt_h = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    mask_h = rng.uniform(0.405, 1.0, (H, W)).astype(np.float32)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and headline and args.extras:
        cpu = cpu_baseline(tgt_h, mask_h)

    # HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default); the
    # gathers' RCCL streams take queues too, so ask for 8 before HIP starts, and
    # refuse a layout with more collective-carrying streams than queues
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
    acct = stream_accounting(args.streams, distributed, GATHER, int(os.environ["GPU_MAX_HW_QUEUES"]))
    print(f"bench.py: rank {rank}: streams {acct}", file=sys.stderr, flush=True)
    if not acct["ok"]:
        raise SystemExit(f"bench.py: {acct['collective_streams']} streams would carry collectives but "
                         f"GPU_MAX_HW_QUEUES={acct['gpu_max_hw_queues']}: two of them could share a "
                         f"hardware queue and serialise one rank's gathers behind another's")
    wd = Watchdog(rank, world, launch_key())
    wd.arm("set-up (device, target plan, communicators, first barrier)", args.watchdog_init_s)
    import ggs
    from ggs import hip
    lib_mod = getattr(ggs, "_lib", None)
    if os.environ.get("GGS_HIP_RUNTIME") == "system" and hasattr(lib_mod, "rocm_lib_dir"):
        hip_path = ggs.runtime_info().get("hip") or ""
        if os.path.dirname(hip_path) != lib_mod.rocm_lib_dir():
            raise SystemExit(f"bench.py: GGS_HIP_RUNTIME=system but libggs is bound to {hip_path!r} "
                             f"(ggs was imported before the setting took effect)")

    n_dev = ggs.ensure_init()
    if local_rank >= n_dev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local_rank} but only {n_dev} GPU(s) visible")
    hip.set_device(local_rank)
    ggs.select_devices([local_rank])

    pops_h = [synthetic_population(POP, N_SPLATS, 10_000 * rank + i) for i in range(N_POPS)]
    pops = [hip.DeviceArray.from_host(p) for p in pops_h]
    tgt = hip.DeviceArray.from_host(tgt_h)
    mask = hip.DeviceArray.from_host(mask_h)
    outs = [hip.DeviceArray((POP,)) for _ in range(RING)]
    gathered = [hip.DeviceArray((POP * world,)) for _ in range(RING)]
    works = [None] * RING
    assert RING % args.streams == 0, f"--streams must divide {RING}"
    streams = [hip.Stream() for _ in range(args.streams)]
    sts = [s.handle for s in streams]

    # the target/mask are fixed over a GA run: lay them out once for the raster's
    # fitness epilogue (ggs_plan_create), as the device-resident GA does
    plan = ggs.TargetPlan(local_rank, sts[0], tgt.ptr, mask.ptr, ggs.GGS_FIT_WEIGHTED, 1.0, H, W)
    streams[0].synchronize()

    # one RCCL communicator per stream: a communicator orders its collectives
    # across streams, which would serialise the alternating batches again
    comms = [ggs.RcclGather(local_rank) for _ in range(args.streams)] \
        if distributed and GATHER.startswith("rccl") else None

    def join(j):                                             # slot j's stream waits for its gather
        if works[j] is None:
            return
        k, ticket = works[j]
        comms[k].wait(sts[k], ticket)
        works[j] = None

    def step(i, ns, gather=True):
        g, j, k = pops[i % N_POPS], i % RING, i % ns
        st = sts[k]
        wd.step, wd.stream = i, k
        join(j)
        plan.fitness_device(st, g.ptr, POP, N_SPLATS, 9, K_SIGMA, outs[j].ptr)
        if comms is None or not gather:
            return
        # RCCL: fitness scalars to every rank
        works[j] = (k, comms[k].allgather(st, outs[j].ptr, gathered[j].ptr, POP,
                                          overlap=GATHER == "rccl-overlap"))
        wd.collective(k, works[j][1])

    def barrier():
        for j in range(RING):
            join(j)
        for s in streams:
            s.synchronize()
        if comms is not None:
            wd.collective(0)
            comms[0].barrier()
        hip.synchronize()

    # every later phase's deadline: the floor + 20x its expected time at the step
    # time this rank measured alone (the first ramp batch: no collectives)
    t_step = [None]

    def arm(phase, n_steps=0, extra_s=0.0):
        if n_steps and t_step[0] is None:
            # no step time measured yet (--ramp-ms 0): nothing to scale the deadline
            # from, so the set-up's generous deadline applies instead of the bare floor
            wd.arm(phase, max(args.watchdog_init_s, args.watchdog_floor_s + 20.0 * extra_s))
            return
        est = (t_step[0] or 0.0) * n_steps + extra_s
        wd.arm(phase, args.watchdog_floor_s + 20.0 * est)

    # Clock ramp before any measurement: the GPU raises its clocks over tens of ms
    # of load, so run the evaluation untimed for --ramp-ms first (no gathers:
    # ranks may run different numbers of these steps).
    def ramp(ms, ns):
        arm(f"ramp ({ms:.0f} ms, {ns} stream(s))", extra_s=ms * 1e-3)
        t_ramp, i = time.perf_counter(), 0
        while (time.perf_counter() - t_ramp) * 1e3 < ms:
            for _ in range(50):
                step(i, ns, gather=False)
                i += 1
            for s in streams:
                s.synchronize()
            if t_step[0] is None:
                t_step[0] = (time.perf_counter() - t_ramp) / 50
        barrier()

    def max_over_ranks(vals):
        v = np.asarray(vals, np.float64)
        if comms is None:
            return v
        wd.collective(0)
        return comms[0].allgather_host(v.astype(np.float32)).astype(np.float64).max(0)

    def timed(ns):
        """W untimed steps, then passes of exactly K steps, each bracketed by
        barrier + synchronize, until --min-time seconds were measured (the same
        number of passes on every rank).  Returns (median pass seconds after the
        max over ranks per pass, passes, host enqueue seconds of the first pass)."""
        arm(f"warm-up ({args.warmup} steps, {ns} stream(s))", args.warmup)
        for i in range(args.warmup):
            step(i, ns)
        barrier()

        def one_pass():
            arm(f"timed pass ({args.steps} steps, {ns} stream(s))", args.steps)
            t0 = time.perf_counter()
            for i in range(args.steps):
                step(i, ns)
            host_s = time.perf_counter() - t0
            barrier()
            return time.perf_counter() - t0, host_s

        first, host_s = one_pass()
        reps = int(max_over_ranks([min(1000, max(1, math.ceil(args.min_time / max(first, 1e-9))))])[0])
        passes = [first] + [one_pass()[0] for _ in range(reps - 1)]
        per_pass = max_over_ranks(passes)
        return float(np.median(per_pass)), len(passes), host_s

    barrier()                  # first collective's one-time set-up before the ramp, not after it
    ramp(args.ramp_ms, args.streams)
    elapsed, passes, host_s = timed(args.streams)          # the headline
    shard_ok = True
    if comms is not None and GATHER != "none":             # the gather delivered this rank's shard
        j = (args.steps - 1) % RING
        shard_ok = np.array_equal(gathered[j].to_host()[rank * POP:(rank + 1) * POP], outs[j].to_host())

    extras = {}
    kern = {}
    if args.extras:
        # dependent batches (a GA generation needs the previous one's fitness): one stream
        if args.streams > 1:
            ramp(args.ramp_ms / 3, 1)
            elapsed1, passes1, _ = timed(1)
        else:
            elapsed1, passes1 = elapsed, passes
        extras["value_one_stream"] = round(world * POP * args.steps / elapsed1, 1)
        extras["ms_per_step_one_stream"] = round(elapsed1 / args.steps * 1e3, 4)
        # + the D2H of the B fitness scalars each step (fitness.py:42 .cpu()) and a host sync
        ramp(args.ramp_ms / 3, 1)
        host_out = np.empty(POP, np.float32)
        arm("readback passes", extra_s=args.min_time)
        t0 = time.perf_counter()
        n_rb = 0
        while time.perf_counter() - t0 < args.min_time:
            for i in range(args.steps):
                step(i, 1, gather=False)
                hip.memcpy_d2h_async(host_out, outs[i % RING].ptr, POP * 4, streams[0])
                streams[0].synchronize()
            n_rb += args.steps
        rb_s = max_over_ranks([(time.perf_counter() - t0) / n_rb])[0]
        extras["value_with_readback"] = round(world * POP / rb_s, 1)
        barrier()

        # The timed step excludes the target plan (built once above, as the device GA
        # does for its fixed target).  A caller of the plain device API
        # (ggs_fitness_device) rebuilds it on every call: its one-stream rate, and the
        # plan build alone (host-timed around a synchronised ggs_plan_create).
        ramp(args.ramp_ms / 3, 1)
        arm("unplanned device-API passes", extra_s=2 * args.min_time)

        def loop_rate(one):      # seconds per step of one stream, no gathers, same loop shape
            t0, n = time.perf_counter(), 0
            while time.perf_counter() - t0 < args.min_time:
                for i in range(args.steps):
                    one(i)
                streams[0].synchronize()
                n += args.steps
            return (time.perf_counter() - t0) / n
        pl_s = loop_rate(lambda i: step(i, 1, gather=False))
        un_s = loop_rate(lambda i: ggs.fitness_device(local_rank, sts[0], pops[i % N_POPS].ptr, POP, N_SPLATS, 9,
                                                      tgt.ptr, mask.ptr, ggs.GGS_FIT_WEIGHTED, 1.0, H, W,
                                                      K_SIGMA, outs[i % RING].ptr))
        pl_s, un_s = max_over_ranks([pl_s, un_s])
        builds = []
        for _ in range(6):
            t1 = time.perf_counter()
            p2 = ggs.TargetPlan(local_rank, sts[0], tgt.ptr, mask.ptr, ggs.GGS_FIT_WEIGHTED, 1.0, H, W)
            streams[0].synchronize()
            builds.append(time.perf_counter() - t1)
            p2.close()
        extras["plan_excluded"] = {
            "note": "the timed step reuses one target plan (ggs_plan_create, once per target/mask/mode); "
                    "ggs_fitness_device rebuilds it per call",
            "plan_build_ms": round(float(np.median(builds[1:])) * 1e3, 4),
            "device_api_unplanned_value": round(world * POP / un_s, 1),
            "device_api_unplanned_ms_per_step": round(un_s * 1e3, 4),
            "excluded_ms_per_step": round((un_s - pl_s) * 1e3, 4),
            "excluded_rule": "unplanned minus planned one-stream step, both timed in the same loop "
                             "(no gathers, one synchronize per K steps)"}
        barrier()
        ramp(args.ramp_ms / 3, 1)

        # per-kernel device time (HIP events on the launch stream) over a single-stream
        # pass (kernels alone, not sharing the chip with another stream's)
        arm("per-kernel event pass", args.steps)
        ggs.profile_reset()
        ggs.profile_enable(True)
        for i in range(args.steps):
            step(i, 1, gather=False)
        barrier()
        ggs.profile_enable(False)
        kern = {k: ggs.profile_read(k) for k in ("prep", "raster", "finalize")}
    wd.disarm()
    if distributed:
        assert shard_ok, "fitness all-gather returned a different shard"

    # algorithmic work of this workload (AABB pairs from the product's own prep)
    pairs = 0
    for p in pops_h:
        pre = ggs.preprocess(ggs.encode(p), H, W, K_SIGMA)
        pairs += int(((pre["x1"].astype(np.int64) - pre["x0"] + 1) *
                      (pre["y1"].astype(np.int64) - pre["y0"] + 1)).sum())
    pairs_per_cand = pairs / (N_POPS * POP)

    # PCIe-inclusive rate of the host API (numpy genomes in, fitness scalars out:
    # target/mask content check, pinned staging, 3 launches, D2H) — the path a
    # caller handing over host buffers gets; reported beside, never the value
    host_api = None
    if world == 1 and args.extras:
        ggs.fitness(pops_h[0], tgt_h, H, W, K_SIGMA, weight_mask=mask_h, device=local_rank)
        n_h, t_h = 0, time.perf_counter()
        while time.perf_counter() - t_h < 0.5:
            ggs.fitness(pops_h[n_h % N_POPS], tgt_h, H, W, K_SIGMA, weight_mask=mask_h, device=local_rank)
            n_h += 1
        host_api = round(n_h * POP / (time.perf_counter() - t_h), 1)

    total = global_batch * args.steps if scaling == "strong" else world * POP * args.steps
    value = total / elapsed
    ms_step = elapsed / args.steps * 1e3
    step_bytes = bytes_per_candidate() * POP
    roof = None
    if kern:
        raster_ms = kern["raster"][0] / max(kern["raster"][1], 1)
        achieved = step_bytes / (raster_ms * 1e-3) / 1e9
        # PMC figures of a committed profile with this launch's shape (profiles/rNN or
        # rNN_<config>): configs[3] split over 8 ranks launches configs[2]'s 512 per GPU;
        # a --pop exploration has none
        prof_cfg = profile_config(args.config, args.pop, POP)
        kernel = "raster_kernel<1, false, false>" if N_SPLATS <= 512 else "raster_kernel<1, true, false>"
        # PMC figures only from a profile of THIS binary and THIS raster instance
        match, match_why, match_src = profile_match(prof_cfg, kernel, lib_sha256(ggs.LIB_PATH)) \
            if prof_cfg is not None else (False, "no committed profile of this launch shape (--pop)", None)
        profiled = match
        traffic, traffic_src = pmc_traffic(prof_cfg) if profiled else (None, None)
        valu_tflops = FLOP_PER_PAIR * pairs_per_cand * POP / (raster_ms * 1e-3) / 1e12
        busy = pmc_valu_busy(prof_cfg) if profiled else None
        busy_src = match_src if profiled else None
        rp = rocprof_kernel_ms(prof_cfg) if profiled else {}
        ev_sum = sum(v[0] / max(v[1], 1) for v in kern.values())
        # The raster is bound by the VALU: `bound` names
        # that roof.  achieved / peak / frac are the HBM figures the contract defines
        # (algorithmic bytes per launch / HIP-event launch time vs 8 TB/s, frac_roof);
        # the VALU's executed-work fraction is binding_frac (PMC busy).
        roof = {"bound": "valu", "kernel": kernel,
                "profile_match": {"ok": match, "why": match_why, "libggs_sha256": lib_sha256(ggs.LIB_PATH)},
                "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "frac_roof": "hbm",
                "traffic": None if traffic is None else round(traffic),
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": step_bytes,
                "avg_launch_ms": round(raster_ms, 5),
                "regime": "single-stream pass (kernels alone, HIP events on the launch stream); pairs "
                          "with ms_per_step_one_stream, as the committed rocprofv3 trace (bench.py "
                          "--streams 1)",
                "rocprof_trace_avg_ms": (None if not profiled or pmc_trace_avg_us(prof_cfg) is None
                                         else round(pmc_trace_avg_us(prof_cfg) / 1e3, 5)),
                "binding": "valu",
                "binding_frac": busy,
                "step_effective": {"regime": f"headline, {args.streams} streams (overlapping batches)",
                                   "achieved": round(step_bytes / (ms_step * 1e-3) / 1e9, 2),
                                   "frac": round(step_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                                   "ms_per_step": round(ms_step, 5)},
                "note": "VALU/transcendental-bound path (SURVEY.md §8d): see 'valu'"}
        valu = {"frac": busy,
                "frac_definition": "executed VALU issue of the raster kernel: SQ_ACTIVE_INST_VALU x 4 / "
                                   "(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), committed rocprofv3 PMC "
                                   "profile of this launch shape",
                "frac_source": busy_src,
                "reference_equivalent": {
                    "tflops": round(valu_tflops, 3), "fp32_peak_tflops": VALU_PEAK_TFLOPS,
                    "ratio_to_peak": round(valu_tflops / VALU_PEAK_TFLOPS, 4),
                    "flop_per_aabb_pair": FLOP_PER_PAIR, "aabb_pairs_per_candidate": pairs_per_cand,
                    "note": "24 FLOP per AABB pair the reference's per-pixel loop would execute "
                            "(SURVEY.md §8d); the row recurrence executes fewer, so this ratio can "
                            "exceed 1 and is not a roofline fraction"}}
    # what the collective ran on, as RCCL itself reports it (every rank takes part
    # in the host all-gather of (rank, device) pairs), and the runtimes' provenance
    rccl_ranks = rank_devices = None
    if comms:
        n_r, r_r, d_r = comms[0].info()
        rccl_ranks = n_r
        rank_devices = [[int(a), int(b)] for a, b in comms[0].allgather_host([float(r_r), float(d_r)])]
    runtime = ggs.runtime_info()
    if rank == 0:
        line = {
            "metric": METRIC if headline else
            f"candidate renders/sec, {H}x{W}, {N_SPLATS} splats, pop={global_batch}"
            + (f" split over {world} GPU(s)" if scaling == "strong" else f" per GPU x {world}"),
            "value": round(value, 1),
            "unit": "candidate renders/s",
            "value_semantics": (f"throughput of independent populations alternating over {args.streams} "
                                "HIP streams (one batch's grid tail overlaps the next batch); "
                                "value_one_stream is the rate a generation-by-generation caller "
                                "(algorithm.py:123-141: the next generation needs this one's fitness) "
                                "gets, value_with_readback adds the per-step D2H of the fitness scalars"),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (population.py distributions, U[0,1] target, U[0.405,1] mask)",
            "config": {"workload": f"{H}x{W} canvas, {N_SPLATS} splats/candidate, "
                                   + (f"pop={global_batch} split over {world} GPU(s) ({POP} per GPU)"
                                      if scaling == "strong" else f"pop={POP} per GPU")
                                   + ", weighted-L2 fitness (encode+prep+raster+reduce"
                                   + (" + RCCL fitness all-gather)" if comms else ")"),
                       "H": H, "W": W, "splats": N_SPLATS, "pop_per_gpu": POP,
                       "global_batch": global_batch, "parallelism": f"dp{world} (candidate shards)",
                       "fitness_gather": (GATHER if comms else None),
                       "rccl_ranks": rccl_ranks,            # ncclCommCount of this run's communicator
                       "rank_devices": rank_devices},       # [ncclCommUserRank, ncclCommCuDevice] per rank
            "timing": {"passes": passes, "statistic": "median pass of K steps (max over ranks per pass)",
                       "measured_s": round(elapsed * passes, 3)},
            "gsplat_pixels_per_s": round(value * N_SPLATS * H * W / 1e9, 2),
            "aabb_pairs_per_s": round(value * pairs_per_cand, 1),
            "roofline": roof,
            "valu": valu if kern else None,
            "streams": args.streams,
            **extras,
            "host_enqueue_ms_per_step": round(host_s / args.steps * 1e3, 4),
            "host_api_renders_per_s": host_api,
            "kernels_ms_per_launch": {k: round(v[0] / max(v[1], 1), 5) for k, v in kern.items()},
            "kernels_ms_rocprof": (rp or None) if kern else None,
            "kernel_timing_note": (None if not kern else
                                   f"HIP events bracket each launch on its stream (one event pair per kernel): "
                                   f"prep + raster + finalize sum to {ev_sum:.4f} ms against a "
                                   f"{extras.get('ms_per_step_one_stream', float('nan')):.4f}-ms one-stream step, "
                                   f"so each event figure carries the pair's overhead and the launch gap; "
                                   f"kernels_ms_rocprof is the committed trace of the same binary"),
            "hip_runtime": _mapped("libamdhip64"),
            "runtime": runtime,                              # ggs_runtime_info: HIP + RCCL paths, versions, one tree
            "torch_loaded": "torch" in sys.modules,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    # communicator teardown can hang too (an RCCL destroy waits for its peers)
    wd.arm("teardown (communicators)", args.watchdog_floor_s)
    for c in comms or ():
        c.close()
    wd.disarm()
    wd.close()


def _mapped(name):
    try:
        for line in open("/proc/self/maps"):
            if name in line:
                return line.split()[-1]
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
