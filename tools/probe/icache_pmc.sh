#!/bin/bash
# Counter inventory of the box, then instruction-fetch counters of the raster at the
# bench shape (512^2/256/128) and a lone 2048^2/4096 candidate (rtime.py workers).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/icache; export TMPDIR=/tmp
timeout -k 5 120 rocprofv3 --list-avail > gpurun_out/icache/avail.txt 2>&1
grep -o -E "\b(SQ|SQC)_[A-Z0-9_]+" gpurun_out/icache/avail.txt | sort -u > gpurun_out/icache/names.txt
want=""
for c in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES; do
  grep -qx "$c" gpurun_out/icache/names.txt && want="$want $c"
done
echo "counters:$want"
for cfg in 512 sa2; do
  timeout -s KILL 120 rocprofv3 --pmc $want --kernel-include-regex raster_kernel -d gpurun_out/icache/$cfg -o run --output-format csv -- python3 tools/probe/rtime.py --worker --config $cfg --steps 20 --out /tmp/x.npy > gpurun_out/icache/$cfg.log 2>&1 || { echo "pmc $cfg failed"; tail -5 gpurun_out/icache/$cfg.log; exit 1; }
  python3 - "$cfg" <<'PY'
import csv, glob, sys, collections
f = glob.glob(f"gpurun_out/icache/{sys.argv[1]}/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[1], {k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
done
