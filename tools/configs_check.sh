#!/bin/bash
# The other BASELINE configs on the current code, one GPU: configs[2] and configs[3]
# bench lines (single GPU), their single-stream rocprofv3 profiles
# (tools/profile_configs.sh -> gpurun_out/prof_<tag>_1024{,x8}), and the configs[4] SA
# loop at the start of a run and late in it (tools/bench_sa.py, device loop).
#   bash tools/configs_check.sh <round tag, e.g. r04>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${1:-r04}
for c in 1024 1024x8; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${R}_bench_$c.log 2>&1 || exit $?
  grep '^{' gpurun_out/${R}_bench_$c.log | tail -1 > gpurun_out/${R}_bench_$c.json
  python3 -c "import json; d=json.load(open('gpurun_out/${R}_bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['kernels_ms_per_launch'])"
done
bash tools/profile_configs.sh $R > gpurun_out/${R}_profile_configs.log 2>&1 || { tail -5 gpurun_out/${R}_profile_configs.log; exit 1; }
tail -12 gpurun_out/${R}_profile_configs.log
timeout -k 10 400 python3 tools/bench_sa.py --only device_loop_full --repeat 3 > gpurun_out/${R}_sa_start.json 2>&1 || exit $?
tail -1 gpurun_out/${R}_sa_start.json | cut -c1-400
timeout -k 10 400 python3 tools/bench_sa.py --only device_loop_full --repeat 3 --warm 2000 --temp0 1e-6 > gpurun_out/${R}_sa_late.json 2>&1 || exit $?
tail -1 gpurun_out/${R}_sa_late.json | cut -c1-400
