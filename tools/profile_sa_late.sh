#!/bin/bash
# rocprofv3 trace + PMC passes (tools/profile.sh) of the SA device loop late in a run
# (configs[4], --warm 2000 --temp0 1e-6: rounds of 16 neighbours) -> gpurun_out/prof_<tag>.
# The warm-up's narrower rounds are in the same process, so the raster's counters
# and trace average are taken over the width-16 launches only (PROF_RASTER_GRID:
# 16 neighbours x 2,048 strip-waves x 64 threads); tools/pack_profile.sh keeps
# the same rows.  Copy into profiles/ with tools/collect_profile.sh <tag>.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PROF_RASTER_GRID=${PROF_RASTER_GRID:-2097152}
BENCH="python3 tools/bench_sa.py --only device_loop_full --dev-iters 300 --repeat 1 --warm 2000 --temp0 1e-6" \
    bash tools/profile.sh ${1:-r03_sa_late} > /dev/null || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/prof_${1:-r03_sa_late}/summary.json'))
for k, v in sorted(d['kernels'].items(), key=lambda kv: -kv[1]['pct'])[:6]:
    print('  %-58s calls %5d avg %10.1f us %6.1f%%' % (k[:58], v['calls'], v['avg_us'], v['pct']))
c = d['counters']; r = [k for k in c if 'raster' in k]
for k in r:
    x = c[k]; print('  %s VALU busy %.3f' % (k, x['SQ_ACTIVE_INST_VALU'] * 4 / (x['GRBM_GUI_ACTIVE'] / 8 * 1024)))
print('  raster HBM bytes/launch', d['raster_hbm_bytes_per_launch'])
print('  grid filter', d.get('raster_grid_filter'))
"
