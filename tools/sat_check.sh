#!/bin/bash
# Saturation cut-off A/B: GPU parity suite, raster timing at the bench workload,
# configs[2] bench and configs[4] SA with and without the cut-off (GGS_SATURATE=0 build).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
L=genetic-gaussian-splats_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/ablate.py $L/libggs.so $L/libggs_nosat.so
for lib in libggs.so libggs_nosat.so; do
  GGS_LIB=$PWD/$L/$lib timeout -k 10 300 python bench.py --config 1024 --steps 10 --warmup 2 --no-cpu-baseline | grep -o '"value": [0-9.]*' | sed "s/^/$lib 1024: /"
  GGS_LIB=$PWD/$L/$lib timeout -k 10 300 python tools/bench_sa.py --iters 30 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib SA', {k: v['iters_per_s'] for k, v in d.items() if isinstance(v, dict) and 'iters_per_s' in v})"
done
