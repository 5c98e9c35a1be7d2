#!/bin/bash
# SA device loop at configs[4] per libggs build, builds alternated (ALT = libs under the package dir).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd
for i in 1 2 3; do
  for L in libggs ${ALT:-libggs_b256 libggs_b384}; do
    GGS_LIB=$PWD/$P/$L.so timeout -k 10 300 python tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 1 ${SA_ARGS:-} > gpurun_out/sa_ab_$L.$i.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['device_loop_full']; print(sys.argv[2], d['iters_per_s'], d['us_per_round'], d['launches'])" gpurun_out/sa_ab_$L.$i.log $L
  done
done
