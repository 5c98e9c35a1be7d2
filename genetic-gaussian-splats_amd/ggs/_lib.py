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
    "ggs_comm_info": (C.c_int, [C.c_void_p, _i32p, _i32p, _i32p]),
    "ggs_runtime_info": (C.c_int, [C.c_char_p, C.c_int32]),
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


def _torch_lib_dir():
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return None
    if spec is None or not spec.submodule_search_locations:
        return None
    d = os.path.join(list(spec.submodule_search_locations)[0], "lib")
    return d if os.path.exists(os.path.join(d, "libamdhip64.so")) else None


def rocm_lib_dir() -> str:
    """/opt/rocm's library directory ($ROCM_PATH), resolved to its release tree."""
    return os.path.realpath(os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib"))


# the runtime libraries this module loaded by absolute path (kept referenced)
_runtime_handles = []


def _bind_hip_runtime() -> None:
    """One HIP runtime per process, loaded by absolute path before libggs (which
    binds it by SONAME, libamdhip64.so.7, so it takes the one already loaded).
    PyTorch-ROCm wheels bundle their own libamdhip64 under the same SONAME: if
    libggs bound /opt/rocm's copy first, a later ``import torch`` would load a
    second runtime and whichever initialises second finds no GPU.  The
    reference's callers hand us torch tensors, so when torch is installed (not
    necessarily imported) its runtime is the one.  GGS_HIP_RUNTIME=system:
    $ROCM_PATH's (/opt/rocm), by absolute path — a bare SONAME search can resolve
    to torch's copy through the library path (the round-5 bench line ran on it)."""
    if os.environ.get("GGS_HIP_RUNTIME", "") == "system":
        d = rocm_lib_dir()
        names = ("libhsa-runtime64.so.1", "libamdhip64.so.7")
    else:
        d = _torch_lib_dir()
        names = ("libhsa-runtime64.so", "libamdhip64.so")
        if d is None:
            return                      # no torch: libggs's own runpath (/opt/rocm/lib)
    for n in names:
        p = os.path.join(d, n)
        if not os.path.exists(p):
            raise ImportError(f"HIP runtime {p} not found (GGS_HIP_RUNTIME="
                              f"{os.environ.get('GGS_HIP_RUNTIME', '')!r}, ROCM_PATH)")
        _runtime_handles.append(C.CDLL(p, mode=C.RTLD_GLOBAL))


def mapped(name: str):
    """Paths of this process's mapped shared objects whose file name starts with `name`."""
    out = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1]
                if os.path.basename(p).startswith(name) and p not in out:
                    out.append(p)
    except OSError:
        pass
    return out


def preload_rccl() -> None:
    """Load the RCCL of the HIP runtime's tree (its directory: /opt/rocm's or
    PyTorch's bundled one, which torch.distributed uses) by absolute path,
    RTLD_LOCAL, before the first communicator; libggs finds it by SONAME and
    refuses an RCCL from another directory.  RTLD_LOCAL is the fix for the exit
    abort of round 5 (docs/EXPERIMENTS.md §16): PyTorch's librccl exports 223 weak
    libstdc++ template instantiations (std::_Rb_tree<std::string, ...>::_M_erase,
    shared_ptr's _M_release_last_use_cold, ...); loaded RTLD_GLOBAL before
    ``import torch``, the torch libraries loaded later bound those calls to its
    copies (LD_DEBUG=bindings: libtorch_cpu, libtorch_python, libc10, librocfft,
    libhipblaslt, MIOpen, ...) and the interpreter aborted at exit with "double free
    or corruption" — reproduced on a CPU host with no GPU, gone with RTLD_LOCAL."""
    hips = mapped("libamdhip64")
    if len(hips) != 1:
        raise ImportError(f"expected one HIP runtime in the process, found {hips}")
    d = os.path.dirname(os.path.realpath(hips[0]))
    for n in ("librccl.so.1", "librccl.so"):
        p = os.path.join(d, n)
        if os.path.exists(p):
            _runtime_handles.append(C.CDLL(p, mode=C.RTLD_LOCAL))
            return
    # none beside it: libggs reports the failure at the first communicator


def _load() -> C.CDLL:
    _bind_hip_runtime()
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


def runtime_info() -> dict:
    """ggs_runtime_info: the HIP runtime libggs is bound to and the RCCL it loaded
    (paths, versions, one tree or not) — what a run's record names."""
    import json
    need = lib.ggs_runtime_info(None, 0)
    buf = C.create_string_buffer(max(int(need), 1))
    rc = lib.ggs_runtime_info(buf, len(buf))
    if rc != GGS_OK:
        raise GGSError(f"ggs_runtime_info: {rc}")
    return json.loads(buf.value.decode())
