#!/bin/bash
# Copy the judged rocprofv3 summaries of tools/profile.sh <tag> from the scratch
# gpurun_out/prof_<tag>/ into the tracked profiles/<tag>/: the trace's per-kernel
# stats, the summary, the commands, and the counter rows of the raster kernel
# (one row per dispatch and counter; the other kernels' rows are in the summary's
# means).
set -eu
cd "$(dirname "$0")/.."
TAG=${1:-r03}
SRC=gpurun_out/prof_$TAG
[ -d "$SRC" ] || SRC=gpurun_out/pack_$TAG      # packed on the box (tools/pack_profile.sh)
DST=profiles/$TAG
mkdir -p "$DST"
cp "$SRC/trace/run_kernel_stats.csv" "$DST/kernel_stats.csv"
for p in fetch write sq wait; do
    python3 - "$SRC/pmc_$p/run_counter_collection.csv" "$DST/pmc_${p}_raster.csv" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "raster_kernel" in r["Kernel_Name"]]
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Dispatch_Id", "Kernel_Name", "Grid_Size", "VGPR_Count", "SGPR_Count", "LDS_Block_Size",
                "Counter_Name", "Counter_Value", "Duration_ns"])
    for r in rows:
        w.writerow([r["Dispatch_Id"], r["Kernel_Name"].split("(")[0], r["Grid_Size"], r["VGPR_Count"],
                    r["SGPR_Count"], r["LDS_Block_Size"], r["Counter_Name"], r["Counter_Value"],
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"])])
PY
done
cp "$SRC/commands.txt" "$DST/"
# stamp the git revision: only when this tree's libggs.so is the profiled build
python3 - "$SRC/summary.json" "$DST/summary.json" <<'PY'
import hashlib, json, subprocess, sys
d = json.load(open(sys.argv[1]))
st = d.setdefault("stamp", {})
lib = st.get("libggs") or "genetic-gaussian-splats_amd/libggs.so"
mine = hashlib.sha256(open(lib, "rb").read()).hexdigest()
if st.get("libggs_sha256") != mine:
    sys.exit(f"collect_profile: {lib} here ({mine[:16]}) is not the profiled build "
             f"({str(st.get('libggs_sha256'))[:16]}): rebuild from the profiled revision or re-profile")
git = lambda *a: subprocess.run(["git", *a], capture_output=True, text=True).stdout.strip()
st["git_head"] = git("rev-parse", "HEAD")
st["git_tree_dirty"] = bool(git("status", "--porcelain", "--", "genetic-gaussian-splats_amd/csrc", "include"))
json.dump(d, open(sys.argv[2], "w"), indent=1)
PY
echo "copied $SRC -> $DST"
