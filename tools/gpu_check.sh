#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; a crash/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() {  # rc 0 (pass) / 1 (test failures) continue; anything else stops
  local rc=$1 what=$2
  echo "[$what] rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what"; exit "$rc"; fi
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
ok_or_stop $? pytest_gpu
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
ok_or_stop $? smoke
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1
ok_or_stop $? bench
cat gpurun_out/bench.log
