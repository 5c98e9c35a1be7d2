#!/bin/bash
# Round-3 final profiles on the final code: the headline (profiles/r03) and the other
# bench configs (r03_1024, r03_1024x8), each from single-stream passes; then the SA
# loop's late regime FETCH/WRITE (r03_sa_late) and the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 900 bash tools/profile.sh r03 > gpurun_out/profile_r03.log 2>&1; ok_or_stop $? profile_r03
timeout -k 10 900 bash tools/profile_configs.sh r03 > gpurun_out/profile_cfg_r03.log 2>&1; ok_or_stop $? profile_cfg_r03
cat gpurun_out/profile_cfg_r03.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1
ok_or_stop $? bench; tail -1 gpurun_out/bench.log | cut -c1-400
