#!/bin/bash
# A/B of the saturation-cut cull's prefetch depth (GGS_SAT_AHEAD builds) and HEAD:
# raster ms at the bench (non-SAT instance), the lone 2048^2 SA shapes and 1024^2,
# then the SA device loop at configs[4] (start of a run).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd
LIBS=${LIBS:-"$P/libggs.so $P/libggs_ah1.so $P/libggs_head.so"}
for c in ${CFGS:-512 sa2 sa16 1024}; do
  timeout -k 10 400 python tools/probe/rtime.py --config $c --rounds ${ROUNDS:-3} $LIBS > gpurun_out/ah_$c.log 2>&1 || exit $?
  grep SUMMARY gpurun_out/ah_$c.log
done
for L in $LIBS; do
  echo "$L $(GGS_LIB=$PWD/$L timeout -k 10 300 python tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 3 | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["device_loop_full"]; print(d["iters_per_s"], d["runs_iters_per_s"], d["us_per_round"])')" || exit $?
done
