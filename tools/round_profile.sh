#!/bin/bash
# One GPU session that re-takes this round's judged numbers on the current code:
# the default bench line (with the CPU baseline), the headline rocprofv3 trace +
# PMC passes (tools/profile.sh), and the shipped-GA-run rates, profile and
# per-wave timing (tools/ga_default.sh).
#   bash tools/round_profile.sh <round tag, e.g. r04>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04}
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/${TAG}_bench.log | tail -1 > gpurun_out/${TAG}_bench_line.json
cut -c1-300 gpurun_out/${TAG}_bench_line.json
bash tools/profile.sh $TAG > gpurun_out/${TAG}_profile.log 2>&1 || { tail -5 gpurun_out/${TAG}_profile.log; exit 1; }
bash tools/ga_default.sh ${TAG}_ga_default > gpurun_out/${TAG}_ga_default.log 2>&1 || { tail -5 gpurun_out/${TAG}_ga_default.log; exit 1; }
tail -12 gpurun_out/${TAG}_ga_default.log | cut -c1-300
