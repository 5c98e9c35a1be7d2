#!/bin/bash
# kernel trace of the SA loop per lib (LIBS)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
for L in ${LIBS}; do
  mkdir -p gpurun_out/sa_tr_$L
  GGS_LIB=$PWD/genetic-gaussian-splats_amd/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sa_tr_$L -o run --output-format csv -- python3 tools/bench_sa.py --only device_loop_full --dev-iters 100 --repeat 1 > gpurun_out/sa_tr_$L/log.txt 2>&1 || exit $?
done
