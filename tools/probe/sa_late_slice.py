"""Slice a tools/profile_sa_late.sh run down to its timed late-regime rounds: the
last K raster dispatches of each pass (the run's warm-up rounds come first), per
pass the raster rows, and a summary of those rows (VALU busy, fabric bytes per
launch, mean duration).  Writes <dir>_late/ and removes the full per-dispatch
CSVs so the copy-back stays small.

    python tools/probe/sa_late_slice.py gpurun_out/prof_r03_sa_late [K]"""
import csv, json, os, shutil, sys

src = sys.argv[1].rstrip("/")
K = int(sys.argv[2]) if len(sys.argv) > 2 else 100
dst = src + "_late"
os.makedirs(dst, exist_ok=True)


def raster_rows(path):
    rows = [r for r in csv.DictReader(open(path)) if "raster_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0))
    return rows


out = {"last_dispatches": K}
tr = raster_rows(os.path.join(src, "trace", "run_kernel_trace.csv"))[-K:]
out["raster_avg_us"] = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr) / len(tr) / 1e3
cnt = {}
for p in ("fetch", "write", "sq", "wait"):
    f = os.path.join(src, f"pmc_{p}", "run_counter_collection.csv")
    rows = raster_rows(f)
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})[-K:]
    keep = [r for r in rows if int(r["Dispatch_Id"]) in set(ids)]
    with open(os.path.join(dst, f"pmc_{p}_raster_last.csv"), "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["Dispatch_Id", "Grid_Size", "Counter_Name", "Counter_Value"])
        for r in keep:
            w.writerow([r["Dispatch_Id"], r["Grid_Size"], r["Counter_Name"], r["Counter_Value"]])
    for r in keep:
        cnt.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
mean = {k: sum(v) / len(v) for k, v in cnt.items()}
out["counters_mean_per_dispatch"] = mean
out["valu_busy"] = mean["SQ_ACTIVE_INST_VALU"] * 4 / (mean["GRBM_GUI_ACTIVE"] / 8 * 1024)
out["fabric_bytes_per_launch"] = mean["FETCH_SIZE"] * 1024 * 2 + mean["WRITE_SIZE"] * 1024
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
shutil.copy(os.path.join(src, "commands.txt"), os.path.join(dst, "commands.txt"))
json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
shutil.rmtree(src)
print(json.dumps({k: v for k, v in out.items() if k != "counters_mean_per_dispatch"}))
