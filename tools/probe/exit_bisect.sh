#!/bin/bash
# Which GPU test files, run in one process, end in an abort at interpreter exit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
T="python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step() { local tag=$1; shift; timeout -k 10 300 $T "$@" > gpurun_out/bis_$tag.log 2>&1; local r=$?; echo "$tag rc=$r"; [ $r -eq 0 ] || exit $r; }
for s in ${STEPS:?}; do step $s $(echo $s | tr '+' ' ' | sed 's#\([a-z_]*\)#tests/test_gpu_\1.py#g'); done
