#!/bin/bash
# Headline bench at several stream counts, alternated twice (counts must divide bench.py RING;
# the round-2 sweep of 3 and 6 streams ran with RING = 24).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do for s in ${STREAMS_LIST:-2 4 8}; do
  GGS_BENCH_STREAMS=$s timeout -k 10 200 python bench.py --no-cpu-baseline --steps 24 --warmup 6 --extras 0 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('streams $s', d['value'])" || exit $?
done; done
