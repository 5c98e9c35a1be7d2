#!/bin/bash
# A/B of the saturation-cut cull batch (GGS_SAT_BATCH builds libggs_b<N>.so against
# libggs.so = batch CAP): raster ms at the lone-candidate SA shapes and at 1024^2,
# then the SA device loop at configs[4] (start of run) per build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd
LIBS="$P/libggs.so ${ALT:-$P/libggs_b128.so $P/libggs_b192.so $P/libggs_b256.so $P/libggs_b384.so}"
for c in sa2 sa16 1024; do
  timeout -k 10 400 python tools/probe/rtime.py --config $c --rounds 2 $LIBS > gpurun_out/satb_$c.log 2>&1 || exit $?
  grep SUMMARY gpurun_out/satb_$c.log
done
for L in $LIBS; do
  echo "$L $(GGS_LIB=$PWD/$L timeout -k 10 300 python tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 2 | tail -1 | cut -c1-200)" || exit $?
done
