#!/bin/bash
# round 6: this build vs round 5's (libggs_r05.so) — raster A/B at four launch
# shapes and the shipped GA, alternated
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
ALT="libggs_r05 libggs" CFGS="512 ga24 sa2 1024" ROUNDS=3 bash tools/probe/ab_rtime.sh || exit 1
ALT="libggs_r05 libggs" GENS=4000 bash tools/probe/ga_ab.sh || exit 1
