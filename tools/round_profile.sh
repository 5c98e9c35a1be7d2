#!/bin/bash
# The round's judged numbers on the current build, in two GPU sessions (each fits
# gpurun's 20-minute limit):
#   bash tools/round_profile.sh <tag> A   GPU test suite, the default bench line (with
#                                          the CPU baseline), rocprofv3 trace + PMC
#                                          profiles <tag> (headline), <tag>_1024,
#                                          <tag>_1024x8 (configs[2]/[3] launches) and
#                                          <tag>_render (the render API, batch)
#   bash tools/round_profile.sh <tag> B   the shipped GA run (rates x3, profile
#                                          <tag>_ga_default, per-wave timing with the
#                                          probe library if built), the configs[4] SA
#                                          loop at the start of a run and late (rates,
#                                          profiles <tag>_sa and <tag>_sa_late)
# Then, HERE (not on the box): tools/collect_profile.sh <each tag> — it refuses a
# profile whose libggs.so sha256 is not this tree's build and stamps the git head.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:?tag}; PART=${2:?A or B}
ok() { local rc=$1; echo "[$2] rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
show() { python3 - "$1" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["pct"])[:5]:
    print("  %-56s calls %6d avg %9.2f us %5.1f%%" % (k[:56], v["calls"], v["avg_us"], v["pct"]))
st = d.get("stamp", {})
k = st.get("raster_kernel")
if k and k in d["counters"]:
    x = d["counters"][k]
    print("  %s VALU busy %.3f, HBM bytes/launch %s, lib %s" % (k, x["SQ_ACTIVE_INST_VALU"] * 4 / (x["GRBM_GUI_ACTIVE"] / 8 * 1024),
          round(d.get("raster_hbm_bytes_per_launch", {}).get("total", 0)), str(st.get("libggs_sha256"))[:16]))
PY
}
if [ "$PART" = A ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/${TAG}_pytest_gpu.log 2>&1; ok $? pytest_gpu
  tail -2 gpurun_out/${TAG}_pytest_gpu.log
  timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1; ok $? bench
  grep '^{' gpurun_out/${TAG}_bench.log | tail -1 > gpurun_out/${TAG}_bench_line.json
  cut -c1-400 gpurun_out/${TAG}_bench_line.json; echo
  bash tools/profile.sh $TAG > gpurun_out/${TAG}_profile.log 2>&1; ok $? profile_$TAG
  show gpurun_out/prof_$TAG/summary.json
  bash tools/profile_configs.sh $TAG > gpurun_out/${TAG}_profile_configs.log 2>&1; ok $? profile_configs
  for t in ${TAG}_1024 ${TAG}_1024x8; do echo "== $t"; show gpurun_out/prof_$t/summary.json; done
  BENCH="python3 tools/bench_render.py --preset batch --iters 30 --min-time 0.05" PROF_STEPS=30 \
      bash tools/profile.sh ${TAG}_render > gpurun_out/${TAG}_render_profile.log 2>&1; ok $? profile_render
  show gpurun_out/prof_${TAG}_render/summary.json
  for p in batch frame final; do
    timeout -k 10 120 python3 tools/bench_render.py --preset $p > gpurun_out/${TAG}_render_$p.json 2>&1; ok $? render_$p
    tail -1 gpurun_out/${TAG}_render_$p.json | cut -c1-300
  done
elif [ "$PART" = B ]; then
  bash tools/ga_default.sh ${TAG}_ga_default > gpurun_out/${TAG}_ga_default.log 2>&1; ok $? ga_default
  tail -12 gpurun_out/${TAG}_ga_default.log | cut -c1-300
  bash tools/pack_profile.sh ${TAG}_ga_default
  for run in start late; do
    args=""; [ $run = late ] && args="--warm 2000 --temp0 1e-6"
    timeout -k 10 400 python3 tools/bench_sa.py --only device_loop_full --repeat 3 $args > gpurun_out/${TAG}_sa_$run.json 2>&1
    ok $? sa_$run
    tail -1 gpurun_out/${TAG}_sa_$run.json | cut -c1-400; echo
  done
  BENCH="python3 tools/bench_sa.py --only device_loop_full --dev-iters 100 --repeat 1" \
      bash tools/profile.sh ${TAG}_sa > gpurun_out/${TAG}_sa_profile.log 2>&1; ok $? profile_sa
  show gpurun_out/prof_${TAG}_sa/summary.json
  bash tools/pack_profile.sh ${TAG}_sa
  bash tools/profile_sa_late.sh ${TAG}_sa_late > gpurun_out/${TAG}_sa_late_profile.log 2>&1; ok $? profile_sa_late
  show gpurun_out/prof_${TAG}_sa_late/summary.json
  PROF_RASTER_GRID=2097152 bash tools/pack_profile.sh ${TAG}_sa_late
else
  echo "part must be A or B"; exit 2
fi
