#!/bin/bash
# A/B of libggs builds (ALT: libs under the package dir, first = baseline) with
# tools/probe/rtime.py at CFGS (raster ms per launch + bit-compare of the fitness).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd
LIBS=""; for L in ${ALT:-libggs_base libggs}; do LIBS="$LIBS $P/$L.so"; done
for c in ${CFGS:-512 sa2 sa16 1024}; do
  timeout -k 10 400 python tools/probe/rtime.py --config $c --rounds ${ROUNDS:-3} $LIBS > gpurun_out/ab_$c.log 2>&1 || { tail -5 gpurun_out/ab_$c.log; exit 1; }
  grep SUMMARY gpurun_out/ab_$c.log
done
