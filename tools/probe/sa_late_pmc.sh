#!/bin/bash
# SA late-run regime (configs[4], bench_sa --warm 2000 --temp0 1e-6): kernel trace and
# the SQ counters of the raster launches only (--kernel-include-regex keeps the
# counter collection off the 2,000 warm-up iterations' small kernels).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/prof_r02_sa_late; mkdir -p $OUT; export TMPDIR=/tmp
CMD="python3 tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 1 --warm 2000 --temp0 1e-6"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
   --kernel-include-regex raster_kernel -d $OUT/pmc_sq -o run --output-format csv -- $CMD > $OUT/pmc_sq.log 2>&1
rc=$?; echo "pmc_sq rc=$rc"; exit $rc
