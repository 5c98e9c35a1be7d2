#!/bin/bash
# On the GPU box, after tools/profile.sh <tag>: keep only what tools/collect_profile.sh
# copies into profiles/ (the trace's kernel stats, the raster's counter rows, the
# summary, the commands) in gpurun_out/pack_<tag>/, and drop the raw per-dispatch
# CSVs (a long loop's traces exceed what gpurun copies back).
set -eu
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:?tag}
SRC=gpurun_out/prof_$TAG
DST=gpurun_out/pack_$TAG
rm -rf "$DST"; mkdir -p "$DST/trace"
cp "$SRC/trace/run_kernel_stats.csv" "$DST/trace/"
for p in fetch write sq wait; do
    mkdir -p "$DST/pmc_$p"
    python3 - "$SRC/pmc_$p/run_counter_collection.csv" "$DST/pmc_$p/run_counter_collection.csv" <<'PY'
import csv, sys
import os
# the raster rows of the last 1,500 raster dispatches (a late-SA loop profiles
# ~14k; the summary's means were taken over all of them on the box), or with
# PROF_RASTER_GRID only those of that grid size (what the summary averaged)
gf = int(os.environ.get("PROF_RASTER_GRID", "0") or 0)
with open(sys.argv[1]) as f:
    r = csv.DictReader(f)
    fields = r.fieldnames
    rows = [row for row in r if "raster_kernel" in row["Kernel_Name"] and (not gf or int(row["Grid_Size"]) == gf)]
keep = set(sorted({int(row["Dispatch_Id"]) for row in rows})[-1500:])
with open(sys.argv[2], "w", newline="") as g:
    w = csv.DictWriter(g, fieldnames=fields)
    w.writeheader()
    for row in rows:
        if int(row["Dispatch_Id"]) in keep:
            w.writerow(row)
PY
done
cp "$SRC/summary.json" "$SRC/commands.txt" "$DST/"
rm -rf "$SRC"
echo "packed $DST"
