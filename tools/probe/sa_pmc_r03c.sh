#!/bin/bash
# Round 3: re-run the round-2 crashing command on the round-2 code it crashed on
# (commit 55b23d2, rebuilt from git into abl/r02crash by the caller).  Expected to
# crash the host process if the crash was caused by that code: last step.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/prof_r03_sa_cause; mkdir -p $OUT; export TMPDIR=/tmp
cd abl/r02crash
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d ../../$OUT/r02code -o run --output-format csv -- \
   python3 tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 1 --warm 2000 --temp0 1e-6 \
   > ../../$OUT/r02code.log 2>&1
rc=$?; echo "r02code rc=$rc"; grep -v "^[WE]2026" ../../$OUT/r02code.log | tail -12
exit 0
