#!/bin/bash
# rocprofv3 trace + PMC passes (tools/profile.sh) of the device-resident loops on the
# current code: rNN_ga (tools/bench_ga.py --backend device, 512^2/256/pop 128) and
# rNN_sa (tools/bench_sa.py device loop at configs[4], start of a run).
# Copy into profiles/ with tools/collect_profile.sh rNN_ga / rNN_sa.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=${1:-r03}
BENCH="python3 tools/bench_ga.py --backend device --gens 200" bash tools/profile.sh ${R}_ga > /dev/null || exit $?
BENCH="python3 tools/bench_sa.py --only device_loop_full --dev-iters 100 --repeat 1" bash tools/profile.sh ${R}_sa > /dev/null || exit $?
for t in ${R}_ga ${R}_sa; do echo "== $t"; python3 -c "
import json; d=json.load(open('gpurun_out/prof_$t/summary.json'))
for k, v in sorted(d['kernels'].items(), key=lambda kv: -kv[1]['pct'])[:8]:
    print('  %-58s calls %5d avg %10.1f us %6.1f%%' % (k[:58], v['calls'], v['avg_us'], v['pct']))
c = d['counters']; r = [k for k in c if 'raster' in k]
for k in r:
    x = c[k]; print('  %s VALU busy %.3f' % (k, x['SQ_ACTIVE_INST_VALU'] * 4 / (x['GRBM_GUI_ACTIVE'] / 8 * 1024)))
"; done
