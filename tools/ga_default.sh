#!/bin/bash
# The reference's shipped GA run (run_ggs.py:41, modules/config.py:5-11: 512^2 work
# size, 512 splats, pop 32, elite 8 -> 24 offspring evaluated per generation) on the
# device-resident loop: generations/s, per-generation device time (HIP events),
# rocprofv3 trace + PMC passes -> gpurun_out/prof_<tag>, per-wave timing of one
# generation's raster (probe build, libggs_probe.so) -> gpurun_out/<tag>_waves.json.
#   bash tools/ga_default.sh [tag]      (then tools/collect_profile.sh <tag>)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04_ga_default}
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python3 tools/bench_ga.py --preset default --backend device --gens 4000 \
      > gpurun_out/${TAG}_rate$i.json || exit $?
  cat gpurun_out/${TAG}_rate$i.json
done
BENCH="python3 tools/bench_ga.py --preset default --backend device --gens 400 --profile-gens 0" \
    bash tools/profile.sh $TAG > /dev/null || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/prof_$TAG/summary.json'))
for k, v in sorted(d['kernels'].items(), key=lambda kv: -kv[1]['pct'])[:6]:
    print('  %-58s calls %5d avg %8.2f us %6.1f%%' % (k[:58], v['calls'], v['avg_us'], v['pct']))
c = d['counters']
for k in [k for k in c if 'raster' in k]:
    x = c[k]; print('  %s VALU busy %.3f' % (k, x['SQ_ACTIVE_INST_VALU'] * 4 / (x['GRBM_GUI_ACTIVE'] / 8 * 1024)))
"
if [ -f genetic-gaussian-splats_amd/libggs_probe.so ]; then
  GGS_PROBE=1 GGS_LIB=$PWD/genetic-gaussian-splats_amd/libggs_probe.so timeout -k 10 120 \
      python3 tools/probe/wave_timing_cfg.py --size 512 --splats 512 --batch 24 \
      > gpurun_out/${TAG}_waves.json || exit $?
  head -c 1500 gpurun_out/${TAG}_waves.json
fi
