#!/bin/bash
# Quick counter pass over the bench workload (raster kernel focus).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-q}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"; export TMPDIR=/tmp
BENCH="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- $BENCH > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "raster" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:24s} {sum(v)/len(v):16.1f}")
PY
