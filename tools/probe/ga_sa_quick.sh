#!/bin/bash
# GA/SA GPU tests, then device-GA generations/s, SA it/s (start of run) and the
# breed phase clocks (libggs_vt.so) — after a change to the variation / mutation kernels.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ga.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ga.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ga.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/bench_ga.py --backend device --gens 2000 || exit $?
timeout -k 10 300 python tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 3 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['device_loop_full'])" || exit $?
GGS_LIB=$PWD/genetic-gaussian-splats_amd/libggs_vt.so timeout -k 10 120 python tools/probe/breed_timing.py || exit $?
