#!/bin/bash
# Host render API per libggs build, alternated (LIBS under the package dir).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for i in 1 2; do for L in ${LIBS:-libggs}; do echo "== $L $i"
  GGS_HIP_RUNTIME=system GGS_LIB=$PWD/genetic-gaussian-splats_amd/$L.so timeout -k 10 120 python3 tools/probe/render_host_probe.py || exit 1
done; done
