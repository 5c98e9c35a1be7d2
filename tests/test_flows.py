"""End-to-end flows of the reference's drivers through the drop-in modules.

* configs[0] (run_ggs.py: 128x128 target, 32 splats, pop 8, 1 generation) —
  the CPU plumbing: work size, GA with the oracle as evaluator, curves CSV,
  full-resolution rescale of the best genome (run_ggs.py:38-77);
* the same driver on the GPU with frames and the final full-resolution render;
* configs[4] (run_sags.py: 2048^2, 4096 splats, 8 tries per iteration): the
  batched-speculation SA gives exactly the sequential SA's result on the GPU.
"""
from __future__ import annotations

import csv
import os

import numpy as np
import pytest

import ggs_oracle as O
from test_ga import CFG, MAX_S, MIN_S


def test_resize_helpers_match_reference_semantics():
    from modules.resize import choose_work_size, scale_genome_pixels_anisotropic
    assert choose_work_size(128, 128, 128) == (128, 128)
    assert choose_work_size(300, 200, 128) == (128, 85)        # round(200*128/300) = 85.33
    assert choose_work_size(200, 300, 128) == (85, 128)
    assert choose_work_size(1000, 3, 128) == (128, 1)          # max(1, ...)
    assert choose_work_size(3, 1000, 512) == (2, 512)          # round(1.536)
    g = O.synthetic_population(1, 5, 64, 64, seed=0)[0]
    out = scale_genome_pixels_anisotropic(g, sH=2.5, sW=0.75)
    np.testing.assert_array_equal(out[:, 2], g[:, 2] + np.float32(np.log(0.75)))
    np.testing.assert_array_equal(out[:, 3], g[:, 3] + np.float32(np.log(2.5)))
    np.testing.assert_array_equal(out[:, [0, 1, 4, 5, 6, 7, 8]], g[:, [0, 1, 4, 5, 6, 7, 8]])
    assert out is not g


def test_loss_curve_png_contract(tmp_path, capsys):
    """utils.py:85-130's contract: a PNG per call, nothing for an empty path, a
    warning (no file) without values, ValueError for curves of unequal length."""
    pytest.importorskip("matplotlib")
    from ggs.ga import save_loss_curve_png
    out = tmp_path / "sub" / "loss.png"
    save_loss_curve_png({"best": [3.0, 2.0, 1.0], "mean": [4.0, 3.0, 2.5], "empty": []}, str(out), log_y=True)
    assert out.read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"
    save_loss_curve_png({"best": [1.0]}, "")                       # no path: nothing
    none = tmp_path / "none.png"
    save_loss_curve_png({"best": []}, str(none))
    assert not none.exists() and "No values to plot" in capsys.readouterr().out
    with pytest.raises(ValueError):
        save_loss_curve_png({"a": [1.0, 2.0], "b": [1.0]}, str(tmp_path / "bad.png"))


def test_per_individual_operator_drop_ins():
    from modules import genetic, population, utils
    population.seed(1)
    genetic.seed(2)
    H = W = 48
    pop = population.new_population(6, 12, H, W, MIN_S, MAX_S)
    assert pop.shape == (6, 12, 9) and pop.dtype == np.float32
    fits = [3.0, 1.0, 2.0, 0.5, 4.0, 0.5]
    for _ in range(20):
        w = genetic.tournament_selection(list(pop), fits, k=6)
        assert any(np.array_equal(w, p) for p in pop)
    c1, c2 = genetic.crossover_uniform(pop[0], pop[1])
    both = np.stack([pop[0], pop[1]])
    for r in range(12):            # each row comes from one parent, the other child gets the other
        assert {c1[r].tobytes(), c2[r].tobytes()} == {both[0, r].tobytes(), both[1, r].tobytes()}
    m = genetic._ensure_one_true(np.zeros((5, 2), bool))
    assert m.sum() == 1
    x = genetic.mutate_individual(pop[2], False, 3, 10, "cosine", CFG["mut_sigma_max"],
                                  CFG["mut_sigma_min"], 0.2, H, W, MIN_S, MAX_S)
    assert x.shape == (12, 9) and not np.array_equal(x, pop[2])
    lo, hi = np.log(np.float32(MIN_S)), np.log(np.float32(MAX_S * H))
    assert (x[:, 2:4] >= lo).all() and (x[:, 2:4] <= hi).all()
    y = pop[3].copy()
    y[:, 0] = 2.0
    y[:, 4] = 7.0
    utils.clamp_genome(y, H, W, MIN_S, MAX_S)
    assert (y[:, 0] == 1.0).all() and (np.abs(y[:, 4]) <= np.pi + 1e-6).all()
    assert utils._anneal_factor(5, 10, "linear") == 0.5
    assert utils.build_mut_sigma(10, 10, "cosine", CFG["mut_sigma_max"],
                                 CFG["mut_sigma_min"])["xy"] == pytest.approx(0.01)


def test_config0_run_ggs_plumbing_cpu(tmp_path):
    """configs[0]: run_ggs.py's flow at 128x128 / 32 splats / pop 8 / 1 generation with
    the reference's ELITE_K=8 (= pop: no offspring survive, algorithm.py:140)."""
    from modules.algorithm import genetic_approx
    from modules.resize import choose_work_size, scale_genome_pixels_anisotropic
    from ggs.mask import compute_importance_mask, prepare_target
    H_out, W_out = 150, 140
    target = np.random.default_rng(0).uniform(0, 1, (H_out, W_out, 3)).astype(np.float32)
    H, W = choose_work_size(H_out, W_out, max_side=128)
    assert (H, W) == (128, 119)
    t = prepare_target(target, H, W)
    m = compute_importance_mask(t, H, W, smooth=3, strength=0.7)
    n_eval = []

    def evaluate(G):
        n_eval.append(len(G))
        return O.fitness_many(list(G), t, H, W, 3.0, weight_mask=m).astype(np.float32)

    csv_path = os.path.join(tmp_path, "ga_loss.csv")
    best, best_fit = genetic_approx(target, H, W, "cuda", 8, 32, 1, 2, 8, 0.05, 0.05,
                                    CFG["mut_sigma_max"], CFG["mut_sigma_min"], "cosine", MIN_S,
                                    MAX_S, 3.0, 0.7, False, loss_csv_path=csv_path, seed=42,
                                    evaluate=evaluate, progress=False)
    # elite_k 8 >= pop 8: no offspring survive (algorithm.py:140), so after the
    # initial population nothing is evaluated
    assert n_eval == [8] and best.shape == (32, 9)
    rows = list(csv.reader(open(csv_path)))
    assert rows[0] == ["gen", "best", "mean", "median"] and len(rows) == 3
    assert float(rows[2][1]) == best_fit <= float(rows[1][1])
    full = scale_genome_pixels_anisotropic(best, sH=H_out / float(H), sW=W_out / float(W))
    img = O.render(O.genome_to_renderer_batched(full[None]), H_out, W_out)[0]
    assert img.shape == (H_out, W_out, 3) and 0.0 <= img.min() and img.max() <= 1.0


@pytest.mark.gpu
def test_run_ggs_flow_on_gpu(tmp_path):
    import torch
    from modules.algorithm import genetic_approx
    from modules.encode import genome_to_renderer
    from modules.render import _DEV, render_splats_rgb_triton
    from modules.resize import choose_work_size, scale_genome_pixels_anisotropic
    H_out, W_out = 150, 140
    target = torch.from_numpy(np.random.default_rng(0).uniform(0, 1, (H_out, W_out, 3))
                              .astype(np.float32))
    H, W = choose_work_size(H_out, W_out, max_side=128)
    vid = os.path.join(tmp_path, "frames")
    os.makedirs(vid)
    best, best_fit = genetic_approx(target, H, W, _DEV, 8, 32, 4, 2, 2, 0.05, 0.05,
                                    CFG["mut_sigma_max"], CFG["mut_sigma_min"], "cosine", MIN_S,
                                    MAX_S, 3.0, 0.7, False, save_video=True, frame_every=2,
                                    video_dir=vid, prefix="ga", seed=42, progress=False)
    assert sorted(os.listdir(vid)) == ["ga_0.png", "ga_2.png", "ga_4.png"]
    assert isinstance(best, torch.Tensor) and np.isfinite(best_fit)
    full = scale_genome_pixels_anisotropic(best.to(_DEV), sH=H_out / float(H), sW=W_out / float(W))
    final = render_splats_rgb_triton(genome_to_renderer(full).unsqueeze(0), H_out, W_out,
                                     k_sigma=3.0, device=_DEV, tile=32)[0]
    ref = O.render(O.genome_to_renderer_batched(full.cpu().numpy()[None]), H_out, W_out)[0]
    np.testing.assert_allclose(final.cpu().numpy(), ref, atol=1e-4, rtol=0)


@pytest.mark.gpu
def test_config4_sa_speculation_equals_sequential_on_gpu():
    """configs[4] shape: 2048^2, 4096 splats, 8 tries per iteration."""
    from ggs import annealing as A
    from ggs import ga
    H = W = 2048
    target = np.random.default_rng(3).uniform(0, 1, (H, W, 3)).astype(np.float32)
    init = O.synthetic_population(1, 4096, H, W, seed=5)[0]
    outs = []
    for spec, backend in ((1, "host"), (None, "host"), (None, "device")):
        outs.append(A.simulated_annealing(
            target, H, W, "cuda", n_splats=4096, mutpb=0.05, mut_sigma_max=CFG["mut_sigma_max"],
            mut_sigma_min=CFG["mut_sigma_min"], sigma_schedule="cosine", min_scale_splats=MIN_S,
            max_scale_splats=MAX_S, k_sigma=3.0, mask_strength=0.7, boost_only=False,
            iterations=3, temp0=1e-3, temp_schedule="cosine", tries_per_iter=8,
            init_individual=init, progress=False, return_state=True, speculate=spec,
            backend=backend, draws=ga.NumpyDraws(9)))
    (b1, f1, s1), (b2, f2, s2), (b3, f3, s3) = outs
    np.testing.assert_array_equal(b1, b2)
    np.testing.assert_array_equal(b1, b3)
    assert f1 == f2 == f3 and s1["curves"] == s2["curves"] == s3["curves"]
    assert s1["stats"]["launches"] == 24 and s2["stats"]["launches"] <= 24
    assert s2["stats"]["evaluated"] >= 24
    c = s1["curves"]["best"]
    assert len(c) == 4 and all(b <= a for a, b in zip(c, c[1:]))
