#!/bin/bash
# Device GA at the shipped shape (bench_ga.py --preset default) per libggs build,
# builds alternated (ALT: libs under the package dir).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd
for i in 1 2 3; do
  for L in ${ALT:-libggs}; do
    GGS_LIB=$PWD/$P/$L.so timeout -k 10 200 python3 tools/bench_ga.py --preset default --backend device \
        --gens ${GENS:-4000} > gpurun_out/ga_ab_$L.$i.json 2>&1 || { tail -5 gpurun_out/ga_ab_$L.$i.json; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['device_us_per_gen'], d['best_fit'])" gpurun_out/ga_ab_$L.$i.json $L
  done
done
