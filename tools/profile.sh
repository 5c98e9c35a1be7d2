#!/bin/bash
# rocprofv3 passes over a workload (default: the bench, 512x512 / 256 splats / pop 128):
#   1. --kernel-trace --stats           -> per-kernel durations
#   2. --pmc FETCH_SIZE                 -> HBM read bytes   (own pass)
#   3. --pmc WRITE_SIZE                 -> HBM write bytes  (own pass)
#   4. --pmc SQ_* GRBM_GUI_ACTIVE       -> instruction mix / VALU activity
# Outputs under gpurun_out/prof_<tag>/ plus a summary JSON (tools/prof_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# the profiled command (default: the bench workload); another config:
#   BENCH="python3 bench.py --config 1024 --steps 10 --warmup 2 --no-cpu-baseline" PROF_STEPS=10 tools/profile.sh r01_1024
BENCH=${BENCH:-"python3 bench.py --streams 1 --steps 30 --warmup 5 --min-time 0.05 --ramp-ms 100 --no-cpu-baseline --extras 0"}
export BENCH                     # tools/prof_summary.py stamps the command
run() { local name=$1; shift; echo "== $name: $*" | tee -a "$OUT/commands.txt"; timeout -k 10 300 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/$name.log"; exit $rc; }; }
run trace rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $BENCH
run pmc_fetch rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- $BENCH
run pmc_write rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- $BENCH
run pmc_sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc_sq" -o run --output-format csv -- $BENCH
run pmc_wait rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d "$OUT/pmc_wait" -o run --output-format csv -- $BENCH
case "$BENCH" in *bench.py*) export PROF_BENCH_PASS=1 ;; *) export PROF_BENCH_PASS=0 ;; esac
python3 tools/prof_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
