"""Minimal HIP runtime plumbing over ctypes: device memory, streams, events.

The drop-in path needs no PyTorch (BASELINE.json north_star): callers with
host arrays use the host API (``ggs.fitness`` / ``ggs.render``), and callers
that keep inputs resident in HBM — ``bench.py``, the sharded evaluation, the
tools — allocate them here.  Binds the HIP runtime libggs.so itself uses (its
SONAME, already loaded by ``ggs._lib``), so pointers, streams and events are
shared with the library.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib  # noqa: F401  (loads libggs.so and, through it, the HIP runtime)
from ._lib import GGSError

_hip = C.CDLL("libamdhip64.so.7")
_SIGS = {
    "hipGetDeviceCount": [C.POINTER(C.c_int)],
    "hipSetDevice": [C.c_int],
    "hipGetDevice": [C.POINTER(C.c_int)],
    "hipMalloc": [C.POINTER(C.c_void_p), C.c_size_t],
    "hipFree": [C.c_void_p],
    "hipMemcpy": [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int],
    "hipMemcpyAsync": [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p],
    "hipMemsetAsync": [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p],
    "hipStreamCreateWithFlags": [C.POINTER(C.c_void_p), C.c_uint],
    "hipStreamDestroy": [C.c_void_p],
    "hipStreamSynchronize": [C.c_void_p],
    "hipDeviceSynchronize": [],
    "hipEventCreate": [C.POINTER(C.c_void_p)],
    "hipEventDestroy": [C.c_void_p],
    "hipEventRecord": [C.c_void_p, C.c_void_p],
    "hipEventSynchronize": [C.c_void_p],
    "hipEventElapsedTime": [C.POINTER(C.c_float), C.c_void_p, C.c_void_p],
    "hipGetErrorString": [C.c_int],
}
for _n, _a in _SIGS.items():
    _f = getattr(_hip, _n)
    _f.argtypes = _a
    _f.restype = C.c_char_p if _n == "hipGetErrorString" else C.c_int

H2D, D2H, D2D = 1, 2, 3
STREAM_NON_BLOCKING = 1


def _ck(rc: int, what: str) -> None:
    if rc != 0:
        raise GGSError(f"{what}: {_hip.hipGetErrorString(rc).decode()} (hip error {rc})")


def device_count() -> int:
    n = C.c_int(0)
    rc = _hip.hipGetDeviceCount(C.byref(n))
    return n.value if rc == 0 else 0


def set_device(d: int) -> None:
    _ck(_hip.hipSetDevice(int(d)), "hipSetDevice")


def synchronize() -> None:
    _ck(_hip.hipDeviceSynchronize(), "hipDeviceSynchronize")


class DeviceArray:
    """A float32/int32 device allocation on the current device (``ptr`` is the
    device address handed to the libggs device-pointer API)."""

    def __init__(self, shape, dtype=np.float32):
        self.shape = tuple(int(s) for s in np.atleast_1d(shape)) if not isinstance(shape, tuple) \
            else tuple(int(s) for s in shape)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        p = C.c_void_p()
        _ck(_hip.hipMalloc(C.byref(p), max(self.nbytes, 4)), "hipMalloc")
        self.ptr = p.value

    @classmethod
    def from_host(cls, a: np.ndarray) -> "DeviceArray":
        a = np.ascontiguousarray(a)
        d = cls(a.shape, a.dtype)
        if a.nbytes:
            _ck(_hip.hipMemcpy(C.c_void_p(d.ptr), a.ctypes.data_as(C.c_void_p), a.nbytes, H2D), "hipMemcpy H2D")
        return d

    def to_host(self, stream: "Stream | None" = None) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        if self.nbytes:
            if stream is not None:
                stream.synchronize()
            _ck(_hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr), self.nbytes, D2H),
                "hipMemcpy D2H")
        return out

    def free(self) -> None:
        if getattr(self, "ptr", None):
            _hip.hipFree(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001 — interpreter shutdown
            pass


class Stream:
    """A non-blocking HIP stream (``handle`` is the hipStream_t as an int)."""

    def __init__(self):
        s = C.c_void_p()
        _ck(_hip.hipStreamCreateWithFlags(C.byref(s), STREAM_NON_BLOCKING), "hipStreamCreateWithFlags")
        self.handle = s.value

    def synchronize(self) -> None:
        _ck(_hip.hipStreamSynchronize(C.c_void_p(self.handle)), "hipStreamSynchronize")

    def close(self) -> None:
        if getattr(self, "handle", None):
            _hip.hipStreamDestroy(C.c_void_p(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class Event:
    def __init__(self):
        e = C.c_void_p()
        _ck(_hip.hipEventCreate(C.byref(e)), "hipEventCreate")
        self.handle = e.value

    def record(self, stream: Stream) -> None:
        _ck(_hip.hipEventRecord(C.c_void_p(self.handle), C.c_void_p(stream.handle)), "hipEventRecord")

    def elapsed_ms(self, end: "Event") -> float:
        _ck(_hip.hipEventSynchronize(C.c_void_p(end.handle)), "hipEventSynchronize")
        ms = C.c_float(0.0)
        _ck(_hip.hipEventElapsedTime(C.byref(ms), C.c_void_p(self.handle), C.c_void_p(end.handle)),
            "hipEventElapsedTime")
        return float(ms.value)

    def close(self) -> None:
        if getattr(self, "handle", None):
            _hip.hipEventDestroy(C.c_void_p(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def memcpy_d2h_async(host: np.ndarray, dev_ptr: int, nbytes: int, stream: Stream) -> None:
    """Enqueue a device-to-host copy into ``host`` (which must stay alive until
    the stream has passed it; pageable memory makes the copy synchronous-ish)."""
    _ck(_hip.hipMemcpyAsync(host.ctypes.data_as(C.c_void_p), C.c_void_p(dev_ptr), int(nbytes), D2H,
                            C.c_void_p(stream.handle)), "hipMemcpyAsync D2H")
