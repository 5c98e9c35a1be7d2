#!/bin/bash
# One GPU session that re-takes a round's judged numbers on the current code:
# the GPU test suite, the default bench line (with the CPU baseline), the
# headline rocprofv3 trace + PMC passes (tools/profile.sh), the shipped-GA-run
# rates, profile and per-wave timing (tools/ga_default.sh), and the breed
# kernel's phase clocks at the shipped and bench shapes (probe build).
#   bash tools/round_profile.sh <round tag, e.g. r04> [skip-tests]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04}
if [ "${2:-}" != skip-tests ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -20 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest_gpu.log
fi
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/${TAG}_bench.log | tail -1 > gpurun_out/${TAG}_bench_line.json
cut -c1-300 gpurun_out/${TAG}_bench_line.json
bash tools/profile.sh $TAG > gpurun_out/${TAG}_profile.log 2>&1 || { tail -5 gpurun_out/${TAG}_profile.log; exit 1; }
bash tools/ga_default.sh ${TAG}_ga_default > gpurun_out/${TAG}_ga_default.log 2>&1 || { tail -5 gpurun_out/${TAG}_ga_default.log; exit 1; }
tail -12 gpurun_out/${TAG}_ga_default.log | cut -c1-300
if [ -f genetic-gaussian-splats_amd/libggs_probe.so ]; then
  for shape in "32 512" "128 256"; do
    set -- $shape
    P=$1 N=$2 GGS_PROBE=1 GGS_LIB=$PWD/genetic-gaussian-splats_amd/libggs_probe.so timeout -k 10 120 \
        python tools/probe/breed_timing.py > gpurun_out/${TAG}_breed_P$1_N$2.txt 2>&1 || exit 1
    echo "breed P=$1 N=$2"; cat gpurun_out/${TAG}_breed_P$1_N$2.txt
  done
fi
