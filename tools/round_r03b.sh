#!/bin/bash
# Round-3 (second session) GPU check on the restored tree: parity tests, smoke,
# the bench line, then the SA loop at configs[4] in both regimes (the baseline
# of the per-round fold).  Each step has its own limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
j() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({k: d.get(k) for k in sys.argv[1:]}))" "$@"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
ok_or_stop $? pytest_gpu; tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
ok_or_stop $? smoke; tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1
ok_or_stop $? bench; tail -1 gpurun_out/bench.log | cut -c1-300
if [ "${SA:-1}" = "1" ]; then
  timeout -k 10 300 python tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 3 > gpurun_out/sa_start.log 2>&1
  ok_or_stop $? sa_start; tail -1 gpurun_out/sa_start.log | j device_loop_full
  timeout -k 10 600 python tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 3 --warm 2000 --temp0 1e-6 > gpurun_out/sa_late.log 2>&1
  ok_or_stop $? sa_late; tail -1 gpurun_out/sa_late.log | j device_loop_full
fi
