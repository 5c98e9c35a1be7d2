#!/bin/bash
# Folded SA rounds: the GA/SA GPU tests, then the SA loop at configs[4] in both regimes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
j() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])['device_loop_full']; print({k: d[k] for k in ('iters_per_s','runs_iters_per_s','accepted','launches','evaluated','us_per_round')})"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_ga.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ga.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ga.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 3 | j || exit $?
timeout -k 10 600 python tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 3 --warm 2000 --temp0 1e-6 | j || exit $?
