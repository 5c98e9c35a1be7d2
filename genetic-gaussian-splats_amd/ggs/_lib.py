"""ctypes binding of libggs.so (C ABI declared in include/ggs.h).

The product path is this library and nothing else: if libggs.so is missing or
cannot be loaded, importing ``ggs`` raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("GGS_LIB", os.path.join(_PKG_ROOT, "libggs.so"))

GGS_OK, GGS_EINVAL, GGS_ENODEV, GGS_EHIP, GGS_ENOMEM = 0, -1, -2, -3, -4
GGS_FIT_NONE, GGS_FIT_WEIGHTED, GGS_FIT_BOOST = 0, 1, 2

_f32p = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)
_f64p = C.POINTER(C.c_double)


class GaConfig(C.Structure):
    """ggs_ga_config (include/ggs.h)."""
    _fields_ = [("pop_size", C.c_int32), ("n_splats", C.c_int32), ("H", C.c_int32),
                ("W", C.c_int32), ("tour_k", C.c_int32), ("elite_k", C.c_int32),
                ("cxpb", C.c_float), ("mutpb", C.c_float), ("k_sigma", C.c_float),
                ("min_scale_splats", C.c_float), ("max_scale_splats", C.c_float),
                ("scale_log_lo", C.c_float), ("scale_log_hi", C.c_float),
                ("fitness_mode", C.c_int32), ("boost_beta", C.c_float), ("schedule", C.c_int32),
                ("sig_max", C.c_double * 6), ("sig_min", C.c_double * 6), ("seed", C.c_uint64)]


class GaDraws(C.Structure):
    """ggs_ga_draws (include/ggs.h)."""
    _fields_ = [("tour_idx", _i32p), ("perm", _i32p), ("cx", _i32p), ("cx_u", _f32p),
                ("u_xy", _f32p), ("u_ab", _f32p), ("u_t", _f32p), ("u_rgb", _f32p),
                ("u_a", _f32p), ("k_color", _i32p), ("k_xy", _i32p), ("k_ab", _i32p),
                ("k_t", _i32p), ("n_xy", _f32p), ("n_ab", _f32p), ("n_t", _f32p),
                ("n_rgba", _f32p), ("swap_i", _i32p), ("swap_pick", _i32p), ("swap_u", _f64p)]


# name -> (restype, argtypes); mirrors include/ggs.h one-for-one
SIGNATURES = {
    "ggs_version": (C.c_char_p, []),
    "ggs_init": (C.c_int, [C.c_int32]),
    "ggs_device_count": (C.c_int, []),
    "ggs_select_devices": (C.c_int, [_i32p, C.c_int32]),
    "ggs_last_error": (C.c_char_p, []),
    "ggs_shutdown": (None, []),
    "ggs_render": (C.c_int, [_f32p, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                             C.c_float, _f32p, _f32p, C.c_int32]),
    "ggs_fitness": (C.c_int, [_f32p, C.c_int64, C.c_int32, C.c_int32, _f32p, _f32p, C.c_int32,
                              C.c_float, C.c_int32, C.c_int32, C.c_float, _f32p, C.c_int32]),
    "ggs_encode": (C.c_int, [_f32p, C.c_int64, C.c_int32, _f32p]),
    "ggs_preprocess": (C.c_int, [_f32p, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_float,
                                 _f32p, _i32p]),
    "ggs_render_device": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32,
                                    C.c_int32, C.c_int32, C.c_int32, C.c_float, _f32p, C.c_void_p]),
    "ggs_fitness_device": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32,
                                     C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.c_float,
                                     C.c_int32, C.c_int32, C.c_float, C.c_void_p]),
    "ggs_detmath_eval": (C.c_int, [C.c_int32, _f32p, _f32p, C.c_int64, _f32p]),
    "ggs_profile_enable": (C.c_int, [C.c_int32]),
    "ggs_profile_read": (C.c_int, [C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "ggs_profile_reset": (None, []),
    "ggs_plan_create": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                  C.c_float, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "ggs_fitness_device_planned": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                                             C.c_int32, C.c_int32, C.c_float, C.c_void_p]),
    "ggs_plan_destroy": (None, [C.c_void_p]),
    "ggs_ga_create": (C.c_int, [C.c_int32, C.POINTER(GaConfig), _f32p, _f32p, _f32p,
                                C.POINTER(C.c_void_p)]),
    "ggs_ga_step": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(GaDraws)]),
    "ggs_ga_run": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32]),
    "ggs_ga_read": (C.c_int, [C.c_void_p, _f32p, _f32p, _f32p, _f64p, _f64p, _i32p]),
    "ggs_ga_destroy": (None, [C.c_void_p]),
    "ggs_sa_create": (C.c_int, [C.c_int32, C.POINTER(GaConfig), _f32p, _f32p, _f32p,
                                C.POINTER(C.c_void_p), _f32p]),
    "ggs_sa_propose": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                 C.POINTER(GaDraws), _f32p]),
    "ggs_sa_commit": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    "ggs_sa_read": (C.c_int, [C.c_void_p, _f32p, _f32p, _f32p]),
    "ggs_sa_destroy": (None, [C.c_void_p]),
    "ggs_sa_set_incremental": (C.c_int, [C.c_void_p, C.c_int32]),
    "ggs_sa_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "ggs_sa_run": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                             C.POINTER(C.c_double), C.c_int32, C.POINTER(C.c_double)]),
    "ggs_sa_rounds_per_sync": (C.c_int64, [C.c_int64, C.c_int32]),
    "ggs_sa_loop_state": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                    C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_uint64)]),
    "ggs_sa_accept_uniform": (C.c_int, [C.c_uint64, C.c_int32, C.c_int32, C.POINTER(C.c_double)]),
    "ggs_comm_unique_id": (C.c_int, [C.c_void_p]),
    "ggs_comm_create": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                  C.POINTER(C.c_void_p)]),
    "ggs_comm_allgather": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                                     C.c_int32, C.POINTER(C.c_int64)]),
    "ggs_comm_wait": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64]),
    "ggs_comm_size": (C.c_int, [C.c_void_p, _i32p, _i32p]),
    "ggs_comm_destroy": (None, [C.c_void_p]),
    "ggs_ga_set_comm": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ggs_comm_init_local": (C.c_int, [C.c_int32, _i32p, C.POINTER(C.c_void_p)]),
    "ggs_comm_init_loopback": (C.c_int, [C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "ggs_comm_allgather_host": (C.c_int, [C.c_void_p, _f32p, _f32p, C.c_int64]),
    "ggs_comm_barrier": (C.c_int, [C.c_void_p]),
}


class GGSError(RuntimeError):
    """A libggs call failed (HIP runtime error, allocation failure, ...)."""


class GGSDeviceError(GGSError, AssertionError):
    """No usable HIP device — the reference's ``assert dev.type == "cuda"``
    (render.py:217) raises AssertionError; this subclasses it as well."""


class GGSInputError(AssertionError, ValueError):
    """Bad argument.  The reference reports these through ``assert``
    (render.py:219, :223), hence the AssertionError base; ValueError too."""


def _share_hip_runtime_with_torch() -> None:
    """One HIP runtime per process.  PyTorch-ROCm wheels bundle their own
    libamdhip64 (same SONAME as /opt/rocm's).  If libggs binds /opt/rocm's copy
    first, a later ``import torch`` loads a second runtime and whichever
    initialises second finds no GPU.  The reference's callers hand us torch
    tensors, so when torch is installed (not necessarily imported) its runtime is
    loaded first (RTLD_GLOBAL) and libggs binds to it by SONAME.
    GGS_HIP_RUNTIME=system skips this."""
    if os.environ.get("GGS_HIP_RUNTIME", "") == "system":
        return
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if spec is None or not spec.submodule_search_locations:
        return
    tlib = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    hip = os.path.join(tlib, "libamdhip64.so")
    if os.path.exists(hip):
        for dep in ("libhsa-runtime64.so", "libamdhip64.so"):
            p = os.path.join(tlib, dep)
            if os.path.exists(p):
                C.CDLL(p, mode=C.RTLD_GLOBAL)


def preload_rccl() -> None:
    """Same rule for RCCL (ggs_comm_*): PyTorch bundles its own librccl with the
    SONAME of /opt/rocm's, so libggs's dlopen must find the copy torch.distributed
    uses.  Called before the first communicator is made.  torch itself is imported
    here, not just its librccl: a process that initialised RCCL and imported torch
    only afterwards aborted at interpreter exit ("double free or corruption", after
    every call had returned; tools/probe/exit_bisect.sh: tests/test_gpu_comm.py then
    test_gpu_parity.py's torch tests), while torch imported first never did."""
    if os.environ.get("GGS_HIP_RUNTIME", "") == "system":
        return
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return
    if spec is None or not spec.submodule_search_locations:
        return
    try:
        import torch  # noqa: F401  (loads its librccl as well)
        return
    except Exception:  # noqa: BLE001 — a broken torch install: bind its librccl only
        pass
    p = os.path.join(list(spec.submodule_search_locations)[0], "lib", "librccl.so")
    if os.path.exists(p):
        C.CDLL(p, mode=C.RTLD_GLOBAL)


def _load() -> C.CDLL:
    _share_hip_runtime_with_torch()
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libggs.so not found at {LIB_PATH}: build it with "
            f"`make -C {os.path.join(_PKG_ROOT, 'csrc')}` (or __graft_entry__.build()). "
            "There is no CPU fallback.")
    lib = C.CDLL(LIB_PATH)
    # an older build loaded for an A/B timing (GGS_LIB=libggs_<rev>.so) may lack
    # entry points added since; the in-tree product library must have all of them
    alt = "GGS_LIB" in os.environ and os.path.basename(LIB_PATH) != "libggs.so"
    for name, (res, args) in SIGNATURES.items():
        if alt and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # a diagnostic build (csrc/Makefile `make probe`: per-wave clocks, a plan-less
    # traffic probe with wrong fitness, knob overrides) is never the product
    kind = (lib.ggs_version() or b"").decode()
    if "probe build" in kind and os.environ.get("GGS_PROBE") != "1":
        raise ImportError(f"{LIB_PATH} is a diagnostic probe build ({kind}); set GGS_PROBE=1 to load it "
                          "for a measurement tool, never for results")
    return lib


lib = _load()
_init_lock = threading.Lock()


def last_error() -> str:
    msg = lib.ggs_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> None:
    if rc == GGS_OK:
        return
    msg = f"{what}: {last_error()}"
    if rc == GGS_EINVAL:
        raise GGSInputError(msg)
    if rc == GGS_ENODEV:
        raise GGSDeviceError(msg)
    raise GGSError(f"{msg} (code {rc})")


# The C library's device list (ggs_select_devices) is process-wide state: the
# host API selects its call's devices and makes the call under this lock, and
# ``selected`` mirrors what was last handed to the library by anyone.
device_lock = threading.RLock()
selected = [None]


def select_devices(ids) -> int:
    """Restrict the host API to these HIP device ids (empty: all)."""
    ensure_init()
    ids = tuple(int(i) for i in ids)
    arr = (C.c_int32 * max(len(ids), 1))(*ids)
    with device_lock:
        selected[0] = None                    # unknown until the call succeeds
        rc = lib.ggs_select_devices(arr, len(ids))
        if rc < 0:
            check(rc, "ggs_select_devices")
        selected[0] = ids
    return rc


def ensure_init() -> int:
    """Initialise every visible HIP device once; returns the device count."""
    with _init_lock:
        n = lib.ggs_device_count()
        if n > 0:
            return n
        rc = lib.ggs_init(0)
        if rc < 0:
            check(rc, "ggs_init")
        return rc
