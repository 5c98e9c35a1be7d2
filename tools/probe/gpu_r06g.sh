#!/bin/bash
# round 6: breed stores staged through LDS — GA tests, soak digests, A/B vs the build before
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ga.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/g_ga.log 2>&1
rc=$?; tail -3 gpurun_out/g_ga.log; [ $rc -eq 0 ] || exit $rc
SOAK_GENS=100000 timeout -k 10 200 python tools/probe/fold_soak.py > gpurun_out/g_soak.log 2>&1 || exit 1
tail -1 gpurun_out/g_soak.log
SOAK_SHAPE=bench SOAK_GENS=20000 timeout -k 10 200 python tools/probe/fold_soak.py > gpurun_out/g_soak_bench.log 2>&1 || exit 1
tail -1 gpurun_out/g_soak_bench.log
ALT="libggs_base libggs" bash tools/probe/ga_ab.sh || exit 1
