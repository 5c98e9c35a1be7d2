#!/bin/bash
# rtime.py A/B of libggs builds over several configs + bitcmp.py, on the GPU box:
#   CFGS="512 ga24 sa1 sa2" LIBS="libggs libggs_x" bash tools/probe/ab_cfgs.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd
L=""; for x in ${LIBS:-libggs}; do L="$L $P/$x.so"; done
for c in ${CFGS:-512 ga24 sa1 sa2}; do
  timeout -k 10 300 python3 tools/probe/rtime.py --config $c --rounds ${ROUNDS:-3} $L > gpurun_out/ab_$c.log 2>&1 \
      || { tail -5 gpurun_out/ab_$c.log; exit 1; }
  grep SUMMARY gpurun_out/ab_$c.log
done
timeout -k 10 300 python3 tools/probe/bitcmp.py $L
