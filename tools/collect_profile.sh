#!/bin/bash
# Copy the judged rocprofv3 summaries of tools/profile.sh <tag> from the scratch
# gpurun_out/prof_<tag>/ into the tracked profiles/<tag>/.
set -eu
cd "$(dirname "$0")/.."
TAG=${1:-r01}
SRC=gpurun_out/prof_$TAG
DST=profiles/$TAG
mkdir -p "$DST"
cp "$SRC/trace/run_kernel_stats.csv" "$DST/kernel_stats.csv"
for p in fetch write sq wait; do
    cp "$SRC/pmc_$p/run_counter_collection.csv" "$DST/pmc_${p}_counters.csv"
done
cp "$SRC/summary.json" "$SRC/commands.txt" "$DST/"
echo "copied $SRC -> $DST"
