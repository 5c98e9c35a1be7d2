#!/bin/bash
# round 6: GPU suite on the build, then the visit-word raster vs the build before it (libggs_base)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t4.log 2>&1
rc=$?; tail -3 gpurun_out/t4.log; [ $rc -eq 0 ] || exit $rc
ALT="libggs_base libggs" CFGS="512 ga24" ROUNDS=5 bash tools/probe/ab_rtime.sh || exit 1
P=genetic-gaussian-splats_amd
for i in 1 2 3; do for L in libggs_base libggs; do
  GGS_LIB=$PWD/$P/$L.so timeout -k 10 120 python3 tools/bench_render.py --preset batch > gpurun_out/render_ab_$L.$i.json 2>&1 || { tail -3 gpurun_out/render_ab_$L.$i.json; exit 1; }
  echo "$L $i $(tail -1 gpurun_out/render_ab_$L.$i.json | cut -c1-160)"
done; done
