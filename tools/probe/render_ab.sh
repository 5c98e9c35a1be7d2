#!/bin/bash
# Render API (tools/bench_render.py) per libggs build, builds alternated
# (ALT: libs under the package dir), presets in PRESETS.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd
for i in 1 2 3; do
  for pre in ${PRESETS:-batch}; do
    for L in ${ALT:-libggs}; do
      GGS_LIB=$PWD/$P/$L.so timeout -k 10 120 python3 tools/bench_render.py --preset $pre > gpurun_out/render_ab_$L.$pre.$i.json 2>&1 \
          || { tail -5 gpurun_out/render_ab_$L.$pre.$i.json; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['preset'], d['renders_per_s'], d['kernels_ms_per_launch'])" gpurun_out/render_ab_$L.$pre.$i.json $L
    done
  done
done
