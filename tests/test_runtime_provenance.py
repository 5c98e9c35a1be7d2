"""One ROCm tree per process (HIP runtime + RCCL), and the exit abort of round 5
pinned at its cause — CPU tests: loading libraries needs no GPU.

* libggs binds the HIP runtime ggs/_lib.py loads by absolute path (PyTorch's
  bundled copy, or /opt/rocm's with GGS_HIP_RUNTIME=system) and loads RCCL only
  from that runtime's directory; an RCCL from anywhere else is refused.
* The abort: PyTorch's librccl, loaded RTLD_GLOBAL before ``import torch``, had
  torch's libraries bind libstdc++ template code to its copies, and the
  interpreter died at exit with "double free or corruption".  preload_rccl loads
  it RTLD_LOCAL (docs/EXPERIMENTS.md §16)."""
from __future__ import annotations

import os
import subprocess
import sys
import textwrap

import pytest

from conftest import PKG

TORCH_LIB = None
try:
    import importlib.util
    _spec = importlib.util.find_spec("torch")
    if _spec and _spec.submodule_search_locations:
        TORCH_LIB = os.path.join(list(_spec.submodule_search_locations)[0], "lib")
except (ImportError, ValueError):
    pass


def _run(code, env=None, timeout=240):
    e = dict(os.environ)
    e.pop("GGS_HIP_RUNTIME", None)
    e.update(env or {})
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], env=e, capture_output=True, text=True,
                          timeout=timeout)


needs_torch_rccl = pytest.mark.skipif(not (TORCH_LIB and os.path.exists(os.path.join(TORCH_LIB, "librccl.so"))),
                                      reason="PyTorch-ROCm with a bundled librccl not installed")


@needs_torch_rccl
def test_rccl_then_torch_exits_cleanly():
    """The round-5 sequence — RCCL initialised (a communicator id made), torch
    imported only afterwards — now exits with status 0."""
    r = _run(f"""
        import sys, ctypes as C
        sys.path.insert(0, {PKG!r})
        import ggs
        from ggs import _lib
        _lib.preload_rccl()
        b = (C.c_uint8 * 128)()
        assert ggs.lib.ggs_comm_unique_id(b) == 0, _lib.last_error()
        info = ggs.runtime_info()
        assert info["same_tree"] is True and info["rccl_version"] > 0, info
        import torch
        print("ok")
        """)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stderr[-1500:])
    assert "double free" not in r.stderr and "free()" not in r.stderr


@needs_torch_rccl
def test_global_rccl_before_torch_is_the_abort():
    """The cause, isolated from libggs: PyTorch's librccl loaded RTLD_GLOBAL ahead
    of torch aborts the interpreter at exit; RTLD_LOCAL (what preload_rccl does)
    exits cleanly."""
    code = f"""
        import ctypes as C, os
        C.CDLL(os.path.join({TORCH_LIB!r}, "librccl.so"), mode=C.RTLD_{{mode}})
        import torch
        print("imported")
        """
    local = _run(code.format(mode="LOCAL"))
    assert local.returncode == 0, local.stderr[-1500:]
    glob = _run(code.format(mode="GLOBAL"))
    if glob.returncode == 0:
        pytest.skip("this torch build no longer aborts with a global librccl")
    assert glob.stdout.strip() == "imported" and ("double free" in glob.stderr or "free()" in glob.stderr), \
        (glob.returncode, glob.stderr[-1500:])


def test_system_runtime_is_one_rocm_tree():
    """GGS_HIP_RUNTIME=system: the HIP runtime is /opt/rocm's release tree, loaded
    by absolute path (the round-5 bench line had resolved the SONAME to torch's
    copy), and RCCL comes from the same directory."""
    rocm = os.path.realpath(os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib"))
    if not os.path.exists(os.path.join(rocm, "librccl.so.1")):
        pytest.skip("no /opt/rocm RCCL")
    r = _run(f"""
        import sys, json, ctypes as C
        sys.path.insert(0, {PKG!r})
        import ggs
        from ggs import _lib
        before = ggs.runtime_info()
        _lib.preload_rccl()
        b = (C.c_uint8 * 128)()
        rc = ggs.lib.ggs_comm_unique_id(b)     # /opt/rocm's RCCL needs a GPU for the id: the load is the point
        assert rc == 0 or "tree" not in _lib.last_error(), _lib.last_error()
        print("J:" + json.dumps([before, ggs.runtime_info(), _lib.mapped("libamdhip64"), _lib.mapped("librccl")]))
        """, env={"GGS_HIP_RUNTIME": "system"})
    assert r.returncode == 0, r.stderr[-1500:]
    import json
    line = [x for x in r.stdout.splitlines() if x.startswith("J:")][-1]
    before, after, hips, rccls = json.loads(line[2:])
    assert before["rccl"] is None and before["same_tree"] is None
    assert os.path.dirname(after["hip"]) == rocm and os.path.dirname(after["rccl"]) == rocm
    assert after["same_tree"] is True and after["rccl_version"] > 0 and after["hip_version"] > 0
    assert len(hips) == 1 and len(rccls) == 1, (hips, rccls)


_FAKE_RCCL = r"""
typedef int r_t;
r_t ncclGetUniqueId(void* u) { return 0; }
r_t ncclCommInitRank(void* c, int n, char id[128], int r) { return 0; }
r_t ncclAllGather(const void* s, void* d, unsigned long n, int t, void* c, void* st) { return 0; }
r_t ncclCommDestroy(void* c) { return 0; }
r_t ncclCommInitAll(void* c, int n, const int* d) { return 0; }
r_t ncclGroupStart(void) { return 0; }
r_t ncclGroupEnd(void) { return 0; }
const char* ncclGetErrorString(r_t r) { return "fake"; }
r_t ncclGetVersion(int* v) { *v = 99999; return 0; }
r_t ncclCommCount(void* c, int* n) { *n = 1; return 0; }
r_t ncclCommUserRank(void* c, int* r) { *r = 0; return 0; }
r_t ncclCommCuDevice(void* c, int* d) { *d = 0; return 0; }
"""


def test_rccl_from_another_tree_is_refused(tmp_path):
    """An RCCL that is not in the HIP runtime's directory ($GGS_RCCL pointing
    elsewhere: a stub library here) is refused at first use, naming both paths."""
    src = tmp_path / "fake_rccl.c"
    src.write_text(_FAKE_RCCL)
    so = tmp_path / "librccl.so.1"
    subprocess.run(["gcc", "-shared", "-fPIC", "-Wl,-soname,librccl.so.1", "-o", str(so), str(src)], check=True,
                   timeout=120)
    r = _run(f"""
        import sys, ctypes as C
        sys.path.insert(0, {PKG!r})
        import ggs
        from ggs import _lib
        b = (C.c_uint8 * 128)()
        rc = ggs.lib.ggs_comm_unique_id(b)
        print(rc, _lib.last_error())
        """, env={"GGS_RCCL": str(so)})
    assert r.returncode == 0, r.stderr[-1500:]
    out = r.stdout.strip().splitlines()[-1]
    assert out.startswith("-2 ") and "not from the HIP runtime's tree" in out and str(tmp_path) in out, out
