#!/bin/bash
# rocprofv3 summaries of the other BASELINE configs (per config):
#   r02_1024  configs[2]/[3] shard: bench.py --config 1024 (1024^2, 1024 splats, pop 512)
#   r02_ga    device-resident GA at 512^2/256/pop 128 (tools/bench_ga.py --backend device)
#   r02_sa    configs[4] SA: 2048^2, 4096 splats, 8 tries, device loop (tools/bench_sa.py)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
BENCH="python3 bench.py --config 1024 --steps 10 --warmup 2 --no-cpu-baseline" PROF_STEPS=10 \
    bash tools/profile.sh r02_1024 > /dev/null || exit $?
BENCH="python3 tools/bench_ga.py --backend device --gens 200" PROF_STEPS=200 \
    bash tools/profile.sh r02_ga > /dev/null || exit $?
BENCH="python3 tools/bench_sa.py --only device_loop_full --dev-iters 100 --repeat 1" PROF_STEPS=100 \
    bash tools/profile.sh r02_sa > /dev/null || exit $?
for t in r02_1024 r02_ga r02_sa; do echo "== $t"; python3 -c "
import json,sys; d=json.load(open('gpurun_out/prof_$t/summary.json'))
for k,v in d['kernels'].items(): print(f'  {k[:60]:60s} calls {v[\"calls\"]:6d} avg {v[\"avg_us\"]:10.1f} us  {v[\"pct\"]:5.1f}%')
print('  raster HBM bytes/launch', d.get('raster_hbm_bytes_per_launch', {}).get('total'))"; done
