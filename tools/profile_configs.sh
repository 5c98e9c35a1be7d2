#!/bin/bash
# rocprofv3 summaries of the other BASELINE configs (per config), each
# from a single-stream bench pass (--streams 1), so a kernel's trace average is its
# exclusive per-launch time (no overlap with another stream's launches):
#   rNN_1024    configs[2] (and configs[3]'s per-GPU launch at 8 ranks): bench.py --config 1024
#               (1024^2, 1024 splats, pop 512)
#   rNN_1024x8  configs[3] at N = 1: bench.py --config 1024x8 (pop 4096 in one launch)
# TAG prefix: $1 (default r03).  GA / SA profiles: tools/profile_ga_sa.sh.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=${1:-r03}
BENCH="python3 bench.py --config 1024 --streams 1 --steps 10 --warmup 2 --min-time 0.05 --ramp-ms 100 --no-cpu-baseline --extras 0" PROF_STEPS=10 \
    bash tools/profile.sh ${R}_1024 > /dev/null || exit $?
BENCH="python3 bench.py --config 1024x8 --streams 1 --steps 2 --warmup 1 --min-time 0.05 --ramp-ms 100 --no-cpu-baseline --extras 0" PROF_STEPS=2 \
    bash tools/profile.sh ${R}_1024x8 > /dev/null || exit $?
for t in ${R}_1024 ${R}_1024x8; do echo "== $t"; python3 -c "
import json,sys; d=json.load(open('gpurun_out/prof_$t/summary.json'))
for k,v in d['kernels'].items(): print(f'  {k[:60]:60s} calls {v[\"calls\"]:6d} avg {v[\"avg_us\"]:10.1f} us  {v[\"pct\"]:5.1f}%')
print('  raster HBM bytes/launch', d.get('raster_hbm_bytes_per_launch', {}).get('total'))"; done
