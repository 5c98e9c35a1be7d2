#!/bin/bash
# configs[4] SA loop (2048^2, 4096 splats, 8 tries): full re-render vs the dirty-strip
# path, at the start of a run and late (--warm 2000, T0 1e-6), for both dirty-splat
# rules (GGS_SA_DIRTY_RULE 1 = raster record differs, 0 = genes differ).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for run in start late; do
  args=""; [ $run = late ] && args="--warm 2000 --temp0 1e-6"
  for rule in 1 0; do
    GGS_SA_DIRTY_RULE=$rule timeout -k 10 400 python3 tools/bench_sa.py --only device_loop_full,device_loop_incremental \
        --repeat 3 $args > gpurun_out/sa_dirty_${run}_rule$rule.json 2>&1 || { tail -5 gpurun_out/sa_dirty_${run}_rule$rule.json; exit 1; }
    python3 - gpurun_out/sa_dirty_${run}_rule$rule.json $run $rule <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("device_loop_full", "device_loop_incremental"):
    v = d[k]
    print(sys.argv[2], "rule", sys.argv[3], k, v["iters_per_s"], v["runs_iters_per_s"], "us/round", v["us_per_round"],
          "changed/nb", v["changed_splats_per_neighbour"], "launches", v["launches"], "best", v["best_fit"])
PY
  done
done
