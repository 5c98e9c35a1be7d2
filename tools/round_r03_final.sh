#!/bin/bash
# Round-3 final evidence on the final code: profiles of every bench config
# (profiles/r03, r03_1024, r03_1024x8: single-stream trace + PMC passes), of the
# device GA and SA loops (r03_ga, r03_sa), the section-6 numbers and the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stopping after $what"; exit "$rc"; fi; }
timeout -k 10 900 bash tools/profile.sh r03 > gpurun_out/profile_r03.log 2>&1; ok_or_stop $? profile_r03
timeout -k 10 900 bash tools/profile_configs.sh r03 > gpurun_out/profile_cfg_r03.log 2>&1; ok_or_stop $? profile_cfg_r03
cat gpurun_out/profile_cfg_r03.log
timeout -k 10 900 bash tools/profile_ga_sa.sh r03 > gpurun_out/profile_ga_sa.log 2>&1; ok_or_stop $? profile_ga_sa
cat gpurun_out/profile_ga_sa.log
timeout -k 10 1100 bash tools/probe/numbers.sh > gpurun_out/numbers.log 2>&1; ok_or_stop $? numbers
cut -c1-300 gpurun_out/numbers.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1
ok_or_stop $? bench; tail -1 gpurun_out/bench.log | cut -c1-300
