#!/bin/bash
# Device GA at the shipped shape, one build, an environment switch alternated:
#   ENVS="GGS_GA_PREDRAW=0 GGS_GA_PREDRAW=1" bash tools/probe/ga_env_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2 3; do
  for E in ${ENVS:?}; do
    env $E timeout -k 10 200 python3 tools/bench_ga.py --preset default --backend device \
        --gens ${GENS:-4000} > gpurun_out/ga_env_$E.$i.json 2>&1 || { tail -5 gpurun_out/ga_env_$E.$i.json; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['device_us_per_gen'], d['best_fit'])" gpurun_out/ga_env_$E.$i.json $E
  done
done
