#!/bin/bash
# Host API (ggs.fitness on numpy arrays, 512^2/256/128) per libggs build, alternated:
#   LIBS="libggs_base libggs" bash tools/probe/host_api_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd
for i in 1 2 3; do
  for L in ${LIBS:-libggs}; do
    echo -n "$L $i: "
    GGS_HIP_RUNTIME=system GGS_LIB=$PWD/$P/$L.so timeout -k 10 120 python3 tools/probe/host_api_probe.py 2>&1 | grep "host API" || exit 1
  done
done
