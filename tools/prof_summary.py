"""Summarise a tools/profile.sh run: per-kernel average duration (trace) and
per-launch counter means; HBM traffic per launch with the gfx950 corrections of
MI355X_MICROARCH.md §HBM (FETCH_SIZE reports 1/2 of the bytes of wide streaming
reads -> x2; WRITE_SIZE exact for 16-B streaming stores; both in KiB)."""
import collections, csv, glob, hashlib, json, os, sys

root = sys.argv[1]
out = {"kernels": {}, "counters": {}}
# What was profiled: the library file (sha256; bench.py compares it with the library
# it runs and drops the PMC figures on a mismatch), the command, and below the raster
# kernel's full symbol.  tools/collect_profile.sh adds the git revision (the box has
# no .git) after checking that the tree's own build has this hash.
_repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_lib = os.environ.get("GGS_LIB") or os.path.join(_repo, "genetic-gaussian-splats_amd", "libggs.so")
out["stamp"] = {"libggs": os.path.relpath(_lib, _repo),
                "libggs_sha256": hashlib.sha256(open(_lib, "rb").read()).hexdigest()
                if os.path.exists(_lib) else None,
                "command": os.environ.get("BENCH")}
stats = os.path.join(root, "trace", "run_kernel_stats.csv")
if os.path.exists(stats):
    for r in csv.DictReader(open(stats)):
        out["kernels"][r["Name"].split("(")[0]] = {
            "calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
            "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3,
            "pct": float(r["Percentage"])}
# bench.py's last pass is single-stream with per-launch HIP events (the live
# avg_launch_ms): average the raster over that pass's dispatches alone (the last
# PROF_STEPS).  Only for the bench (tools/profile.sh sets PROF_BENCH_PASS=1 when it
# profiles bench.py); other workloads have no such pass and report the trace average.
trace = os.path.join(root, "trace", "run_kernel_trace.csv")
steps = int(os.environ.get("PROF_STEPS", "30"))
if os.path.exists(trace) and os.environ.get("PROF_BENCH_PASS") == "1":
    rows = [r for r in csv.DictReader(open(trace)) if "raster_kernel" in r.get("Kernel_Name", "")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    if len(dur) >= steps:
        out["raster_profile_pass_avg_us"] = sum(dur[-steps:]) / steps
        out["raster_dispatches"] = len(dur)
# PROF_RASTER_GRID=<threads>: the raster's counters (and a trace average) over the
# dispatches of that grid size only — a loop whose launches vary in width (the SA
# device loop: one grid per round width) is summarised for one width, e.g. the
# late regime's 16-neighbour rounds (16 x 2,048 strip-waves x 64 = 2,097,152)
grid_f = int(os.environ.get("PROF_RASTER_GRID", "0") or 0)


def _grid(r):
    g = r.get("Grid_Size")
    if g is None:
        g = int(r.get("Grid_Size_X", 0) or 0) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)
    return int(g)


agg = collections.defaultdict(lambda: collections.defaultdict(list))
grids_seen = collections.Counter()
for f in glob.glob(os.path.join(root, "pmc_*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if grid_f and "raster_kernel" in k:
            if "sq" in os.path.basename(os.path.dirname(f)) and r["Counter_Name"] == "SQ_WAVES":
                grids_seen[_grid(r)] += 1
            if _grid(r) != grid_f:
                continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
if grid_f:
    tr = os.path.join(root, "trace", "run_kernel_trace.csv")
    durs = []
    if os.path.exists(tr):
        for r in csv.DictReader(open(tr)):
            if "raster_kernel" in r.get("Kernel_Name", "") and _grid(r) == grid_f:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out["raster_grid_filter"] = {
        "grid_threads": grid_f, "strip_waves": grid_f // 64,
        "pmc_dispatches_by_grid_threads": dict(sorted(grids_seen.items())),
        "pmc_dispatches_kept": grids_seen.get(grid_f, 0),
        "trace_dispatches": len(durs),
        "trace_avg_us": (sum(durs) / len(durs)) if durs else None,
        "note": "counters of the raster kernel are means over the dispatches of this grid size only"}
for k, cs in agg.items():
    out["counters"][k] = {c: sum(v) / len(v) for c, v in cs.items()}
rasters = sorted({k for k in list(out["counters"]) + list(out["kernels"]) if "raster_kernel" in k})
out["stamp"]["raster_kernels"] = rasters
out["stamp"]["raster_kernel"] = rasters[0] if len(rasters) == 1 else None
r = next((k for k in out["counters"] if "raster_kernel" in k), None)
if r:
    c = out["counters"][r]
    fetch = c.get("FETCH_SIZE", 0.0) * 1024 * 2          # x2: gfx950 FETCH_SIZE under-count
    write = c.get("WRITE_SIZE", 0.0) * 1024
    out["raster_hbm_bytes_per_launch"] = {"fetch_corrected": fetch, "write": write,
                                          "total": fetch + write,
                                          "raw_FETCH_SIZE_KiB": c.get("FETCH_SIZE"),
                                          "raw_WRITE_SIZE_KiB": c.get("WRITE_SIZE")}
print(json.dumps(out, indent=1))
