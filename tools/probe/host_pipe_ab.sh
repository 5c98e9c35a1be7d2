#!/bin/bash
# Host API (ggs.fitness on numpy arrays, 512^2/256/128): the two-part pipeline
# (GGS_HOST_PIPE=1, default) vs one stream (0), alternated; optional LIBS baseline.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd
for i in 1 2 3; do
  for E in GGS_HOST_PIPE=1 GGS_HOST_PIPE=0; do
    echo -n "$E $i: "
    env $E GGS_HIP_RUNTIME=system timeout -k 10 120 python3 tools/probe/host_api_probe.py 2>&1 | grep "host API" || exit 1
  done
done
