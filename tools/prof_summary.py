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
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "pmc_*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
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
