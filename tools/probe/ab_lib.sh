#!/bin/bash
# A/B of libggs builds on the GPU box: bit-compare each against libggs.so, then
# alternate bench runs (3 rounds).  ALT="libggs_x libggs_y" (names under the package dir).
set -e
cd $GRAFT_REPO_ROOT
ALT=${ALT:-libggs_new}
BENCH_ARGS=${BENCH_ARGS:-"--no-cpu-baseline --steps 200"}
P=genetic-gaussian-splats_amd
for L in $ALT; do
  echo "$L: $(timeout -k 10 300 python tools/probe/bitcmp.py $P/libggs.so $P/$L.so 2>&1 | tail -1)" >> gpurun_out/ab_bitcmp.log
done
for i in 1 2 3; do
 for L in libggs $ALT; do
  GGS_LIB=$PWD/$P/$L.so timeout -k 10 200 python bench.py $BENCH_ARGS > gpurun_out/ab_$L.$i.log 2>&1
 done
done
