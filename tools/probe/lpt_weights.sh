#!/bin/bash
# Cost-model weights of the single-round packing at the shipped GA shape:
#   WEIGHTS="30:7:-1 100:7:-1 1:0:0" bash tools/probe/lpt_weights.sh   (head:pk:add)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in ${ROUNDS:-1 2}; do
  for wt in off ${WEIGHTS:?}; do
    if [ $wt = off ]; then E="GGS_GA_LPT=0"; else IFS=: read h p a <<< "$wt"; E="GGS_GA_LPT=1 GGS_LPT_HEAD=$h GGS_LPT_PK=$p GGS_LPT_ADD=$a"; fi
    env $E timeout -k 10 200 python3 tools/bench_ga.py --preset default --backend device \
        --gens ${GENS:-2000} --profile-gens 400 > gpurun_out/lpt_w_$wt.$i.json 2>&1 || { tail -5 gpurun_out/lpt_w_$wt.$i.json; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['device_us_per_gen']; print(sys.argv[2], d['value'], k['breed_us'], k['raster_us'], k['lpt_us'], d['best_fit'])" gpurun_out/lpt_w_$wt.$i.json $wt
  done
done
