#!/bin/bash
# GA-layer GPU check: the device-GA parity tests, then the shipped-run preset's rate.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ga.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_ga.log 2>&1; rc=$?
tail -4 gpurun_out/pt_ga.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python3 tools/bench_ga.py --preset default --backend device --gens 4000 > gpurun_out/ga_default_$i.json || exit $?
  cat gpurun_out/ga_default_$i.json
done
timeout -k 10 200 python3 tools/bench_ga.py --preset bench --backend device --gens 1000 > gpurun_out/ga_bench.json || exit $?
cat gpurun_out/ga_bench.json
