#!/bin/bash
# Round 3: the round-2 SIGSEGV of ggs_sa_run under rocprofv3 --pmc.
#  1. the SA / comm GPU tests (rounds per host sync now bounded: ggs_sa_rounds_per_sync);
#  2. the exact failing round-2 command (FETCH_SIZE over every kernel), then WRITE_SIZE,
#     committed as profiles/r02_sa_late's missing traffic counters;
#  3. the cause: K fitness evaluations (3 dispatches each) behind one host sync under
#     --pmc, K = 100 then 1,500 (last: it may crash the host process).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/prof_r03_sa_late; mkdir -p $OUT; export TMPDIR=/tmp
CMD="python3 tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 1 --warm 2000 --temp0 1e-6"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ga.py tests/test_gpu_comm.py -m gpu -x -q --timeout 200 \
   --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $CMD > $OUT/pmc_fetch.log 2>&1
rc=$?; echo "pmc_fetch rc=$rc"; tail -2 $OUT/pmc_fetch.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $CMD > $OUT/pmc_write.log 2>&1
rc=$?; echo "pmc_write rc=$rc"; tail -2 $OUT/pmc_write.log; [ $rc -eq 0 ] || exit $rc
for K in 100 1500; do
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/qd$K -o run --output-format csv -- \
     python3 tools/probe/queue_depth_pmc.py $K > $OUT/qd$K.log 2>&1
  rc=$?; echo "queue_depth K=$K rc=$rc"; tail -2 $OUT/qd$K.log; [ $rc -eq 0 ] || exit $rc
done
