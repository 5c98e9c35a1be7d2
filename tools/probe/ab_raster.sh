#!/bin/bash
# A/B of libggs builds on the GPU box: bench.py's value / one-stream value / raster ms
# per build, 2 alternated rounds.  LIBS="libggs libggs_x" (names under the package dir),
# BENCH_ARGS as for bench.py.
cd $GRAFT_REPO_ROOT
P=genetic-gaussian-splats_amd
LIBS=${LIBS:-"libggs"}
BENCH_ARGS=${BENCH_ARGS:-"--no-cpu-baseline"}
for i in 1 2; do
  for L in $LIBS; do
    GGS_LIB=$PWD/$P/$L.so timeout -k 10 200 python bench.py $BENCH_ARGS > gpurun_out/ab_$L.$i.log 2>&1 || { tail -5 gpurun_out/ab_$L.$i.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_$L.$i.log').read().strip().splitlines()[-1]); print('$L', $i, d['value'], d.get('value_one_stream'), d['kernels_ms_per_launch']['raster'])"
  done
done
