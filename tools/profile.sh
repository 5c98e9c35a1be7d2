#!/bin/bash
# rocprofv3 passes over the bench workload: kernel trace + stats, then one PMC
# pass per counter group (never combined with tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline"
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/$name.log"; exit $rc; }; }
run trace rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $BENCH
run pmc_fetch rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- $BENCH
run pmc_write rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- $BENCH
run pmc_valu rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc_valu" -o run --output-format csv -- $BENCH
run pmc_lds rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY -d "$OUT/pmc_lds" -o run --output-format csv -- $BENCH
find "$OUT" -name "*.csv" | head -50
