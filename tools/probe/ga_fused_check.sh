#!/bin/bash
# GA breed check on the GPU box: the GA GPU tests, device-GA generations/s fused vs
# GGS_GA_UNFUSED=1 (2 alternated runs), a kernel trace, and the breed phase clocks
# (libggs_vt.so, tools/probe/breed_timing.py) when that build is present.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ga.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ga.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ga.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python tools/bench_ga.py --backend device --gens 2000 || exit $?
  GGS_GA_UNFUSED=1 timeout -k 10 120 python tools/bench_ga.py --backend device --gens 2000 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ga -o run --output-format csv -- python3 tools/bench_ga.py --backend device --gens 500 > gpurun_out/prof_ga.log 2>&1 || exit $?
if [ -f genetic-gaussian-splats_amd/libggs_vt.so ]; then
  GGS_LIB=$PWD/genetic-gaussian-splats_amd/libggs_vt.so timeout -k 10 120 python tools/probe/breed_timing.py || exit $?
fi
