#!/bin/bash
# Breed kernel time with draws from memory vs Philox (tools/probe/breed_draws_ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
for m in draws philox; do
  OUT=gpurun_out/bd_$m; mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 tools/probe/breed_draws_ab.py --mode $m > $OUT/log.txt 2>&1 || { tail -5 $OUT/log.txt; exit 1; }
  echo "== $m"; grep -h "ga_variation\|raster_kernel<1, false, true>" $(find $OUT -name "*kernel_stats.csv") | cut -d, -f1-5
done
