#!/bin/bash
# round 6: the round-end checks on the final tree — GPU suite, smoke, default bench line
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/final_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/final_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/final_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/final_bench.log 2>&1
rc=$?; tail -1 gpurun_out/final_bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
