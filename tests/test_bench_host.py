"""bench.py's host-side pieces on CPU (no GPU): the workload's algorithmic byte
count, the synthetic population (population.py:20-46
distributions), and where the roofline's PMC traffic / VALU-busy come from."""
from __future__ import annotations

import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_algorithmic_bytes_per_candidate():
    assert (bench.H, bench.W, bench.N_SPLATS) == (512, 512, 256)
    assert bench.bytes_per_candidate() == 4_203_524          # 12HW + 4HW + 36N + 4


def test_synthetic_population_distributions():
    G = bench.synthetic_population(64, 256, 0)
    assert G.shape == (64, 256, 9) and G.dtype == np.float32
    assert (G[..., :2] >= 0).all() and (G[..., :2] <= 1).all()
    lo, hi = np.log(3.0), np.log(0.1 * 512)
    assert (G[..., 2:4] >= lo - 1e-6).all() and (G[..., 2:4] <= hi + 1e-6).all()
    assert (np.abs(G[..., 4]) <= np.pi + 1e-6).all()
    assert (G[..., 5:8] >= 0).all() and (G[..., 5:8] <= 255).all()
    assert (G[..., 8] >= 180).all() and (G[..., 8] <= 255).all()
    # a_log skews small (Beta mean 0.4), b_log large (0.6)
    assert G[..., 2].mean() < G[..., 3].mean()
    np.testing.assert_array_equal(G, bench.synthetic_population(64, 256, 0))


def test_pmc_figures_come_from_this_workloads_profile():
    paths = bench._bench_profiles()
    assert paths and all(os.path.basename(os.path.dirname(p)).startswith("r") for p in paths)
    assert not any("_" in os.path.basename(os.path.dirname(p)) for p in paths)   # not rNN_<config>
    traffic, src = bench.pmc_traffic()
    assert traffic > 0 and src.startswith("profiles/r") and src.endswith("summary.json")
    busy = bench.pmc_valu_busy()
    assert 0.3 < busy < 1.0


def _built_lib():
    return os.path.join(REPO, "genetic-gaussian-splats_amd", "libggs.so")


def test_committed_profiles_are_of_the_shipped_binary():
    """The newest committed profile of each bench config (what bench.py quotes
    traffic, VALU busy and rocprof times from) was taken on exactly the library
    this tree builds (sha256 of libggs.so; the build is reproducible) and names
    exactly the raster instance that config launches — so a kernel change without
    a re-profile fails here, not silently in the bench line (round 4: the
    profiles predated the last raster commit)."""
    import json
    sha = bench.lib_sha256(_built_lib())
    assert sha
    for cfg, kernel in (("512", "raster_kernel<1, false, false>"), ("1024", "raster_kernel<1, true, false>"),
                        ("1024x8", "raster_kernel<1, true, false>")):
        d, src = bench._summary(cfg)
        assert d is not None, cfg
        st = d.get("stamp") or {}
        assert bench._norm_kernel(st.get("raster_kernel")) == kernel, (src, st.get("raster_kernel"))
        assert st.get("libggs_sha256") == sha, (src, "profiled a different libggs.so: re-profile")
        assert st.get("git_head") and st.get("git_tree_dirty") is False, src
        ok, why, _ = bench.profile_match(cfg, kernel, sha)
        assert ok, why
        assert bench.rocprof_kernel_ms(cfg)["raster"] > 0
        json.dumps(d)


def test_profile_mismatch_drops_the_pmc_figures(monkeypatch):
    """A summary of another build or another raster instance is refused with a
    reason (bench.py then reports traffic / binding_frac as null)."""
    d = {"stamp": {"raster_kernel": "void ggs::raster_kernel<1, false, false>", "libggs_sha256": "ab" * 32},
         "counters": {}, "kernels": {}}
    monkeypatch.setattr(bench, "_summary", lambda config="512": (d, "profiles/rXX/summary.json"))
    ok, why, _ = bench.profile_match("512", "raster_kernel<1, false, false>", "cd" * 32)
    assert not ok and "sha256" in why
    ok, why, _ = bench.profile_match("512", "raster_kernel<1, true, false>", "ab" * 32)
    assert not ok and "raster_kernel<1, false, false>" in why
    ok, _, _ = bench.profile_match("512", "raster_kernel<1, false, false>", "ab" * 32)
    assert ok
    d["stamp"] = {}
    assert not bench.profile_match("512", "raster_kernel<1, false, false>", "ab" * 32)[0]


# ---- --gpus N: the rank spawn (no GPU: a stand-in script records what it got) ----
_FAKE_RANK = r'''
import json, os, sys
out = sys.argv[sys.argv.index("--out") + 1]
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
        "GGS_RDZV_KEY")
with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys} | {"argv": sys.argv[1:]}, f)
fail = os.environ.get("FAKE_FAIL_RANK")
sys.exit(3 if fail is not None and fail == os.environ["RANK"] else 0)
'''


def _fake(tmp_path):
    p = tmp_path / "fake_rank.py"
    p.write_text(_FAKE_RANK)
    return str(p)


def test_gpus_flag_spawns_one_process_per_rank(tmp_path):
    import json
    script = _fake(tmp_path)
    rc = bench.spawn_ranks(4, ["--gpus", "4", "--steps", "7", "--out", str(tmp_path)],
                           script=script, gpus_visible=8)
    assert rc == 0
    seen = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(4)]
    assert [s["RANK"] for s in seen] == ["0", "1", "2", "3"]
    assert [s["LOCAL_RANK"] for s in seen] == ["0", "1", "2", "3"]
    assert {s["WORLD_SIZE"] for s in seen} == {"4"} and {s["MASTER_ADDR"] for s in seen} == {"127.0.0.1"}
    assert len({s["MASTER_PORT"] for s in seen}) == 1 and len({s["GGS_RDZV_KEY"] for s in seen}) == 1
    assert all(s["argv"][:4] == ["--gpus", "4", "--steps", "7"] for s in seen)


def test_gpus_flag_failing_rank_fails_the_job(tmp_path, monkeypatch):
    monkeypatch.setenv("FAKE_FAIL_RANK", "1")
    rc = bench.spawn_ranks(2, ["--out", str(tmp_path)], script=_fake(tmp_path), gpus_visible=2)
    assert rc == 3


def test_gpus_flag_more_than_visible_fails_loudly(tmp_path, capsys):
    rc = bench.spawn_ranks(8, ["--out", str(tmp_path)], script=_fake(tmp_path), gpus_visible=1)
    assert rc == 2 and "only 1 GPU" in capsys.readouterr().err
    assert not list(tmp_path.glob("rank*.json"))


def test_gpus_flag_reaches_the_spawn(monkeypatch):
    import pytest
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    got = {}
    monkeypatch.setattr(bench, "spawn_ranks", lambda n, argv, **kw: got.update(n=n, argv=argv) or 0)
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "8", "--steps", "5"])
    assert e.value.code == 0 and got == {"n": 8, "argv": ["--gpus", "8", "--steps", "5"]}


def test_gpus_flag_must_match_the_launchers_world(monkeypatch):
    import pytest
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "1"])
    assert "WORLD_SIZE=2" in str(e.value.code)


def test_strong_scaling_config_splits_the_population():
    H, N, B, scaling = bench.CONFIGS["1024x8"]
    assert (H, N, B, scaling) == (1024, 1024, 4096, "strong")       # BASELINE.json configs[3]
    assert bench.CONFIGS["512"][:3] == (512, 256, 128)               # configs[1]
    assert bench.CONFIGS["1024"][:3] == (1024, 1024, 512)            # configs[2]


def test_visible_gpus_honours_visible_devices_lists(monkeypatch):
    n = bench.visible_gpus()
    if n is None:
        return                                     # no KFD topology here (CPU container)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert bench.visible_gpus() == min(n, 1)


def test_cpu_cores_respects_the_job_share(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.cpu_cores() == min(3, len(os.sched_getaffinity(0)))


def test_profile_config_matches_the_launch_shape():
    assert bench.profile_config("512", 0, 128) == "512"
    assert bench.profile_config("1024", 0, 512) == "1024"
    assert bench.profile_config("1024x8", 0, 4096) == "1024x8"       # N = 1: the whole population
    assert bench.profile_config("1024x8", 0, 512) == "1024"          # N = 8: configs[2]'s launch
    assert bench.profile_config("1024x8", 0, 2048) is None           # N = 2: not profiled
    assert bench.profile_config("512", 64, 64) is None               # --pop exploration


def test_bench_line_names_its_roofs_and_value_semantics(tmp_path):
    """The world-1 JSON line (bench.run on the stand-in GPU of tests/_fakes.py):
    `bound` names the binding roof (VALU), achieved/peak/frac are the HBM figures
    the contract defines (frac_roof), valu.frac is the executed-work PMC busy of
    the committed profile (never the reference-equivalent FLOP ratio, which sits
    under its own name), and the line says that `value` overlaps independent
    batches while value_one_stream is a generation-by-generation caller's rate."""
    import json
    from test_bench_dist import FAST, _run_world
    codes, _, out0 = _run_world(tmp_path, ["--gpus", "1"] + FAST, world=1, slow_rank=None)
    assert codes == [0]
    line = json.loads(out0[0])
    roof, valu = line["roofline"], line["valu"]
    assert roof["bound"] == "valu" and roof["binding"] == "valu" and roof["frac_roof"] == "hbm"
    assert roof["unit"] == "GB/s" and roof["peak"] == bench.HBM_PEAK_GBS
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-4
    busy = bench.pmc_valu_busy()
    assert valu["frac"] == busy == roof["binding_frac"] and 0 < busy < 1
    assert roof["profile_match"]["ok"], roof["profile_match"]
    assert roof["traffic"] and roof["rocprof_trace_avg_ms"] > 0
    assert line["kernels_ms_rocprof"]["raster"] > 0 and "one-stream step" in line["kernel_timing_note"]
    assert valu["frac_source"].startswith("profiles/r") and "SQ_ACTIVE_INST_VALU" in valu["frac_definition"]
    assert "frac" not in valu["reference_equivalent"] and "ratio_to_peak" in valu["reference_equivalent"]
    sem = line["value_semantics"]
    assert "independent populations" in sem and "value_one_stream" in sem and "algorithm.py:123-141" in sem
    assert line["value_one_stream"] > 0 and line["value_with_readback"] > 0
    assert line["config"]["rccl_ranks"] is None and line["n_gpus"] == 1


def test_committed_profile_summaries_agree_with_themselves():
    """Committed profiles/*/summary.json files do not contradict themselves:
    only a bench.py profile (profiles/rNN, rNN_<config>) quotes a single-stream
    profile-pass raster average (raster_profile_pass_avg_us, what the bench line
    pairs with its live HIP-event figure), and that pass is never slower than the
    trace's all-dispatch average beside it (which also holds the overlapped
    multi-stream launches); a GA / SA loop profile has no such pass, so its
    figure is the kernel table's."""
    import glob
    import json
    for p in glob.glob(os.path.join(REPO, "profiles", "*", "summary.json")):
        name = os.path.basename(os.path.dirname(p))
        d = json.load(open(p))
        pass_avg = d.get("raster_profile_pass_avg_us")
        if "_sa" in name or "_ga" in name:
            assert pass_avg is None, p
            continue
        if pass_avg is None:
            continue
        ks = [v["avg_us"] for k, v in d.get("kernels", {}).items() if "raster_kernel" in k]
        assert len(ks) == 1 and pass_avg <= 1.02 * ks[0], (p, pass_avg, ks)
