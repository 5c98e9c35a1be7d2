"""Per-kernel register / scratch / LDS figures of the SHIPPED libggs.so.

Reads the gfx950 code objects embedded in the library's `.hip_fatbin` section
(one clang offload bundle per translation unit) and their AMDHSA metadata notes
(`llvm-readelf --notes`): no GPU, no rebuild, so the figures describe exactly
the binary that runs.  Used by tests/test_kernel_resources.py (the raster must
stay at <= 168 VGPRs, 3 waves/SIMD, no scratch) and by hand:

    python tools/kernel_resources.py [path/to/libggs.so]
"""
from __future__ import annotations

import os
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
# numeric metadata keys kept per kernel (AMDHSA code object v5)
KEYS = ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
        "private_segment_fixed_size", "group_segment_fixed_size", "max_flat_workgroup_size",
        "wavefront_size")


def _code_objects(so_path: str, arch: str) -> list[bytes]:
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "-O", "binary",
                        "--only-section=.hip_fatbin", so_path, fat], check=True)
        blob = open(fat, "rb").read()
    out = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + len(MAGIC))[0]
        off = pos + len(MAGIC) + 8
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", blob, off)
            off += 24
            triple = blob[off:off + tl].decode()
            off += tl
            if triple.endswith(arch) and sz:
                out.append(blob[pos + o:pos + o + sz])
        pos = blob.find(MAGIC, pos + len(MAGIC))
    return out


def _notes(elf: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(elf)
        f.flush()
        return subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name],
                               capture_output=True, text=True, check=True).stdout


def waves_per_simd(vgprs: int) -> int:
    """gfx950: 512 VGPRs per SIMD lane slice, allocated in blocks of 8, <= 8 waves."""
    blocks = max(8, -(-vgprs // 8) * 8)
    return min(8, 512 // blocks)


def _metadata(notes: str) -> list[dict]:
    """The code object's `amdhsa.kernels` list (YAML between `---` and `...`)."""
    import yaml
    start = notes.index("---")
    end = notes.find("\n...", start)
    doc = yaml.safe_load(notes[start:end if end > 0 else None])
    return doc.get("amdhsa.kernels", [])


def kernel_resources(so_path: str, arch: str = "gfx950") -> dict[str, dict[str, int]]:
    """{mangled kernel name: {vgpr_count, sgpr_count, ..., waves_per_simd}}."""
    res: dict[str, dict[str, int]] = {}
    for elf in _code_objects(so_path, arch):
        for k in _metadata(_notes(elf)):
            r = {key: int(k["." + key]) for key in KEYS if "." + key in k}
            r["waves_per_simd"] = waves_per_simd(r["vgpr_count"] + r.get("agpr_count", 0))
            res[k[".name"]] = r
    return res


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names),
                         capture_output=True, text=True, check=True).stdout.splitlines()
    return dict(zip(names, out))


if __name__ == "__main__":
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "genetic-gaussian-splats_amd", "libggs.so")
    r = kernel_resources(so)
    dm = demangle(sorted(r))
    for n in sorted(r):
        v = r[n]
        short = dm[n].split("(")[0]
        print(f"{short:60s} vgpr {v.get('vgpr_count'):4d} sgpr {v.get('sgpr_count'):4d} "
              f"scratch {v.get('private_segment_fixed_size'):4d} spills v{v.get('vgpr_spill_count')}"
              f"/s{v.get('sgpr_spill_count')} lds {v.get('group_segment_fixed_size'):6d} "
              f"waves/SIMD {v.get('waves_per_simd')}")
