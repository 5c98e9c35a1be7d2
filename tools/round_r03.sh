#!/bin/bash
# Round-3 GPU check: parity tests, smoke, bit-compare against the round-2 build,
# the bench line, then the rocprofv3 passes of every config (profiles/r03*).
# Each step has its own limit; a crash/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
ok_or_stop $? pytest_gpu; tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
ok_or_stop $? smoke; tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1
ok_or_stop $? bench; tail -1 gpurun_out/bench.log | cut -c1-400
if [ "${PROFILES:-1}" = "1" ]; then
  timeout -k 10 900 bash tools/profile.sh r03 > gpurun_out/profile_r03.log 2>&1; ok_or_stop $? profile_r03
  timeout -k 10 900 bash tools/profile_configs.sh r03 > gpurun_out/profile_cfg_r03.log 2>&1; ok_or_stop $? profile_cfg_r03
  cat gpurun_out/profile_cfg_r03.log
fi
