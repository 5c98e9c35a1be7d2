#!/bin/bash
# SQ counters of the raster launches per libggs build at an rtime.py config:
#   CFG=sa1 ALT="libggs libggs_x" bash tools/probe/pmc_ab.sh
# pass 1: instruction mix and wave cycles; pass 2: instruction-cache hits/misses.
# Prints per-launch averages (tools/probe/pmc_ab_sum.py).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmc_ab; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd; CFG=${CFG:-sa1}
for L in ${ALT:-libggs}; do
  for pass in 1 2; do
    if [ $pass = 1 ]; then C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
    else C="SQC_ICACHE_MISSES SQC_ICACHE_HITS"; fi
    OUT=gpurun_out/pmc_ab/$L.$CFG.$pass
    GGS_LIB=$PWD/$P/$L.so timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex raster_kernel -d $OUT -o run \
        --output-format csv -- python3 tools/probe/rtime.py --worker --config $CFG --steps 100 --out /tmp/pmc_ab.npy \
        > $OUT.log 2>&1 || { echo "$L pass $pass failed"; tail -5 $OUT.log; exit 1; }
  done
done
python3 tools/probe/pmc_ab_sum.py gpurun_out/pmc_ab
