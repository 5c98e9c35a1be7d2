#!/bin/bash
# A/B of the saturation cut-off variants at configs[2] (1024^2/1024/pop 512) and configs[4] SA.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
L=genetic-gaussian-splats_amd
for rep in 1 2; do
for lib in ${LIBS:-libggs.so libggs_satrows0.so libggs_nosat.so}; do
  GGS_LIB=$PWD/$L/$lib timeout -k 10 300 python bench.py --config 1024 --steps 10 --warmup 2 --no-cpu-baseline | grep -o '"value": [0-9.]*' | sed "s/^/$lib 1024: /"
  GGS_LIB=$PWD/$L/$lib timeout -k 10 300 python tools/bench_sa.py --iters 30 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib SA', {k: v['iters_per_s'] for k, v in d.items() if isinstance(v, dict) and k.startswith('device')})"
done; done
