#!/bin/bash
# Round 3, cause of the round-2 SIGSEGV (ggs_sa_run under rocprofv3 --pmc):
#  1. plain fitness dispatches, K = 5000 evaluations (15,000 dispatches) behind one sync;
#  2. the round-2 command with the rounds-per-sync bound lifted
#     (GGS_SA_MAX_ROUNDS_PER_SYNC=1000000: the round-2 batching rule).
# Step 2 is expected to crash the host process: it is the last step.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/prof_r03_sa_cause; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/qd5000 -o run --output-format csv -- \
   python3 tools/probe/queue_depth_pmc.py 5000 > $OUT/qd5000.log 2>&1
rc=$?; echo "queue_depth K=5000 rc=$rc"; grep -v "^[WE]2026" $OUT/qd5000.log | tail -3; [ $rc -eq 0 ] || exit $rc
export GGS_SA_MAX_ROUNDS_PER_SYNC=1000000
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/unbounded -o run --output-format csv -- \
   python3 tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 1 --warm 2000 --temp0 1e-6 \
   > $OUT/unbounded.log 2>&1
rc=$?; echo "unbounded rc=$rc"; grep -v "^[WE]2026" $OUT/unbounded.log | tail -12
exit 0
