#!/bin/bash
# Fused vs separate finalize (GGS_UNFUSED_FINALIZE=1): GPU parity tests, then
# alternated bench / GA-default runs of the two.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_all.log 2>&1; rc=$?
tail -3 gpurun_out/pt_all.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    GGS_UNFUSED_FINALIZE=$v timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/bench_fin$v.$i.log 2>&1 || exit $?
    python -c "
import json
d=json.loads([x for x in open('gpurun_out/bench_fin$v.$i.log') if x.startswith('{')][-1])
print('unfused=$v', d['value'], d['value_one_stream'], d['value_with_readback'], d['kernels_ms_per_launch'])"
    GGS_UNFUSED_FINALIZE=$v timeout -k 10 200 python3 tools/bench_ga.py --preset default --backend device --gens 4000 > gpurun_out/ga_fin$v.$i.json || exit $?
    python -c "
import json; d=json.load(open('gpurun_out/ga_fin$v.$i.json')); print('unfused=$v GA', d['value'], d['device_us_per_gen'], d['best_fit'])"
  done
done
