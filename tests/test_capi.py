"""The C-ABI boundary on CPU: libggs.so loads, exports exactly what
include/ggs.h declares, the ctypes table matches, and argument validation (the
reference's assert conditions) happens before any device work.  No compute."""
from __future__ import annotations

import inspect
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, REPO

HEADER = os.path.join(REPO, "include", "ggs.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ggs_\w+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("ggs_render", "ggs_fitness", "ggs_render_device", "ggs_fitness_device",
                 "ggs_encode", "ggs_preprocess", "ggs_last_error", "ggs_init"):
        assert must in names


def test_library_exports_every_declared_symbol():
    import ggs
    names = declared_functions()
    out = subprocess.run(["nm", "-D", "--defined-only", ggs.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s+(ggs_\w+)$", out, flags=re.M))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        assert hasattr(ggs.lib, n)


def test_ctypes_table_matches_header():
    from ggs import _lib
    assert sorted(_lib.SIGNATURES) == declared_functions()


def test_version_and_error_string():
    import ggs
    assert b"gfx950" in ggs.lib.ggs_version()
    assert isinstance(ggs.lib.ggs_last_error(), bytes)


def test_input_validation_mirrors_reference_asserts():
    import ggs
    tgt = np.zeros((8, 8, 3), np.float32)
    with pytest.raises(AssertionError):                      # render.py:223
        ggs.fitness(np.zeros((2, 3, 8), np.float32), tgt, 8, 8)
    with pytest.raises(ValueError):                          # render.py:219
        ggs.render(np.zeros((2, 2, 3, 9), np.float32), 8, 8)
    with pytest.raises(ggs.GGSInputError):
        ggs.fitness(np.zeros((2, 3, 9), np.float32), tgt, 8, 9)   # target shape
    # the C layer validates too (before touching a device)
    import ctypes as C
    rc = ggs.lib.ggs_render(None, 1, 1, 8, 4, 4, 3.0, None, None, 0)
    assert rc == -1 and b"9 genome cols" in ggs.lib.ggs_last_error()
    rc = ggs.lib.ggs_fitness(None, 1, 1, 9, None, None, 7, 1.0, 4, 4, 3.0, None, 0)
    assert rc == -1
    rc = ggs.lib.ggs_fitness_device(0, None, None, 1, 1, 9, None, None, 1, 1.0, 4, 4, 3.0, None)
    assert rc == -1 and b"mask" in ggs.lib.ggs_last_error()
    # size limits: the raster's cull list holds 32-bit byte offsets of 64-B records
    # (N * 64 < 2^31), and the grid B * tiles * 4 strips must stay below 2^31
    rc = ggs.lib.ggs_fitness(None, 1, 2**25, 9, None, None, 0, 1.0, 8, 8, 3.0, None, 0)
    assert rc == -1 and b"exceeds the limit" in ggs.lib.ggs_last_error()
    assert ggs.lib.ggs_render(None, 1, 2**25 - 1, 9, 8, 8, 3.0, None, None, 0) != -1 or \
        b"exceeds" not in ggs.lib.ggs_last_error()
    rc = ggs.lib.ggs_render(None, 2**30, 1, 9, 1024, 1024, 3.0, None, None, 0)
    assert rc == -1 and b"grid limit" in ggs.lib.ggs_last_error()
    del C


def test_no_device_is_an_assertion_like_the_reference():
    import ggs
    if ggs.lib.ggs_init(0) > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(AssertionError):                      # render.py:217
        ggs.render(np.zeros((1, 1, 9), np.float32), 4, 4)


# reference signatures (modules/render.py:204-214, fitness.py:8-12, fitness.py:35-39,
# encode.py:4, :28, :63, mask.py:29-38, algorithm.py:17-31) — the drop-ins must accept the
# same parameters (genetic_approx adds keyword-only **hooks: seed, draws, evaluate, ...)
REF_SIGS = {
    ("render", "render_splats_rgb_triton"):
        ["genomes", "H", "W", "*k_sigma=3.0", "*device=None", "*background=(1.0, 1.0, 1.0)",
         "*tile=64", "*num_warps=8", "*num_stages=3", "*use_fp16_canvas=False"],
    ("fitness", "fitness_many"):
        ["pop_batch", "target", "H", "W", "k_sigma", "device", "tile=32", "weight_mask=None",
         "boost_only=False", "boost_beta=1.0"],
    ("fitness", "fitness_population"):
        ["population", "target", "H", "W", "k_sigma", "device", "tile=32", "chunk=None",
         "weight_mask=None", "boost_only=False"],
    ("encode", "axes_angle_to_cholesky"): ["a_log", "b_log", "theta"],
    ("encode", "genome_to_renderer"): ["ind_axes_angle"],
    ("encode", "genome_to_renderer_batched"): ["G_axes"],
    ("algorithm", "genetic_approx"):
        ["target_img_uint8", "H", "W", "device", "pop_size", "n_splats", "generations", "tour_k",
         "elite_k", "cxpb", "mutpb", "mut_sigma_max", "mut_sigma_min", "schedule",
         "min_scale_splats", "max_scale_splats", "k_sigma", "mask_strength", "boost_only",
         "save_video=False", "frame_every=5000", "video_dir=''", "prefix='ga'",
         "loss_png_path=''", "loss_csv_path=''", "loss_log_y=False", "hooks"],
    ("annealing", "simulated_annealing"):
        ["target_img_uint8", "H", "W", "device", "n_splats", "mutpb", "mut_sigma_max",
         "mut_sigma_min", "sigma_schedule", "min_scale_splats", "max_scale_splats", "k_sigma",
         "mask_strength", "boost_only", "iterations", "temp0", "temp_schedule", "tries_per_iter=1",
         "save_video=False", "frame_every=10000", "video_dir=''", "prefix='sa'",
         "loss_png_path=''", "loss_csv_path=''", "loss_log_y=False", "hooks"],
    ("resize", "choose_work_size"): ["Ht", "Wt", "max_side=128"],
    ("resize", "scale_genome_pixels_anisotropic"): ["ind", "sH", "sW"],
    # dtype: numpy's float32 stands in for torch.float32 (no torch in the product path)
    ("population", "sample_log_scales_beta_linear"):
        ["B", "N", "s_lo", "s_hi", "m=0.5", "concentration=8.0", "device='cuda'",
         "dtype=<class 'numpy.float32'>"],
    ("population", "new_population"):
        ["batch_size", "n_splats", "H", "W", "min_scale_splats", "max_scale_splats",
         "device='cuda'", "dtype=<class 'numpy.float32'>"],
    ("population", "new_individual"):
        ["n_splats", "H", "W", "min_scale_splats", "max_scale_splats", "device='cuda'"],
    ("population", "duplicate_individual"): ["ind"],
    ("population", "population_to_list"): ["pop_tensor"],
    ("genetic", "tournament_selection"): ["pop", "fits", "k=2"],
    ("genetic", "crossover_uniform"): ["a", "b", "p=0.5"],
    ("genetic", "_ensure_one_true"): ["mask"],
    ("genetic", "mutate_individual"):
        ["ind", "is_elite", "gen", "total_gens", "schedule", "mut_sigma_max", "mut_sigma_min",
         "mutpb", "H", "W", "min_scale_splats", "max_scale_splats"],
    ("utils", "wrap_angle"): ["theta"],
    ("utils", "_anneal_factor"): ["gen", "total", "kind"],
    ("utils", "build_mut_sigma"): ["gen", "total_gens", "kind", "mut_sigma_max", "mut_sigma_min"],
    ("utils", "clamp_genome"): ["ind", "H", "W", "min_scale_splats", "max_scale_splats"],
    ("utils", "render_axes_angle_to_img"): ["ind_axes_angle", "Hsnap", "Wsnap", "k_sigma", "device"],
    ("utils", "save_frame_png"):
        ["gen", "ind_axes_angle", "pad", "prefix", "video_dir", "H", "W", "k_sigma", "device",
         "save_video=True"],
    ("utils", "prewarm_renderer"): ["H", "W", "k_sigma", "device"],
    ("utils", "save_loss_curve_png"):
        ["curves", "out_path", "title='GA fitness over generations'", "xlabel='Generation'",
         "ylabel='MSE'", "log_y=False", "dpi=144"],
    ("utils", "save_curves_csv"): ["curves", "out_csv_path"],
    ("mask", "compute_importance_mask"):
        ["target_hw3", "H", "W", "edge_scales=(1, 2, 4)", "w_edge=0.7", "w_var=0.3", "gamma=0.7",
         "floor=0.15", "smooth=0", "strength=1.0"],
}


@pytest.mark.parametrize("mod,fn", sorted(REF_SIGS))
def test_drop_in_signatures_match_reference(mod, fn):
    import importlib
    m = importlib.import_module(f"modules.{mod}")
    sig = inspect.signature(getattr(m, fn))
    got = []
    for p in sig.parameters.values():
        s = ("*" if p.kind == p.KEYWORD_ONLY else "") + p.name
        if p.default is not p.empty:
            s += f"={p.default!r}"
        got.append(s)
    assert got == REF_SIGS[(mod, fn)]


def test_drop_in_keeps_module_constant():
    from modules import render
    assert render._DEV == "cuda" and "render_splats_rgb_triton" in render.__all__


def test_package_layout():
    assert os.path.isfile(os.path.join(PKG, "libggs.so"))
    assert os.path.isdir(os.path.join(PKG, "csrc"))


def _build_c_host(tmp_path):
    from ggs import _lib
    exe = os.path.join(tmp_path, "ggs_c_host")
    src = os.path.join(os.path.dirname(__file__), "c", "ggs_c_host.c")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
                    src, "-o", exe, "-L", libdir, "-lggs", "-Wl,-rpath," + libdir, "-lm"],
                   check=True, capture_output=True, text=True)
    return exe


def test_plain_c_host_builds_and_links(tmp_path):
    """A C caller compiles against include/ggs.h alone and links libggs.so; without
    a GPU ggs_init reports GGS_ENODEV (exit 2) — the reference's device assert."""
    import subprocess
    exe = _build_c_host(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode in (0, 2), r.stdout + r.stderr
    assert "ggs" in r.stdout


@pytest.mark.gpu
def test_plain_c_host_fused_fitness_matches_rendered_images(tmp_path):
    import subprocess
    exe = _build_c_host(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("candidate") == 4
