#!/bin/bash
# Headline step time vs streams and batch size (bench.py --streams S --pop P):
# how much of the single-stream raster's fill/tail the overlapping batches recover.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for sp in 1:128 2:128 4:128 8:128 4:256 4:512 8:512 4:1024; do
  s=${sp%%:*}; p=${sp##*:}
  r=$(timeout -k 10 200 python bench.py --streams $s --pop $p --steps 40 --warmup 5 --no-cpu-baseline --extras 0 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('value_one_stream'))") || exit $?
  echo "streams $s pop $p : renders/s ms/step one_stream = $r"
done
