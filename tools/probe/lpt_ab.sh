#!/bin/bash
# Single-round packing A/B at the shipped GA shape (and its raster alone):
# GGS_GA_LPT=1 (default) vs 0, alternated 3x on one box, same library.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2 3; do
  for E in GGS_GA_LPT=1 GGS_GA_LPT=0; do
    env $E timeout -k 10 200 python3 tools/bench_ga.py --preset default --backend device \
        --gens ${GENS:-4000} --profile-gens 400 > gpurun_out/lpt_ab_$E.$i.json 2>&1 || { tail -5 gpurun_out/lpt_ab_$E.$i.json; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['device_us_per_gen'], d['best_fit'])" gpurun_out/lpt_ab_$E.$i.json $E
  done
done
