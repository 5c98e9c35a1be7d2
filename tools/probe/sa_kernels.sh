#!/bin/bash
# GA/SA GPU tests, then the SA device loop at configs[4] (start of run) under a
# kernel trace: per-round kernel averages and the loop's per-round cost.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/sa_k; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ga.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ga.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ga.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 3 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])['device_loop_full']; print({k: d[k] for k in ('iters_per_s','accepted','launches','evaluated','us_per_round','us_per_evaluated')})" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sa_k -o run --output-format csv -- python3 tools/bench_sa.py --only device_loop_full --dev-iters 100 --repeat 1 > gpurun_out/sa_k/log.txt 2>&1 || exit $?
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/sa_k/run_kernel_stats.csv')):
    print(r['Name'][:40].ljust(40), r['Calls'].rjust(6), '%9.2f us' % (float(r['AverageNs']) / 1e3))
"
