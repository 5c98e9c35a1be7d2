#!/bin/bash
# Record-fetch latency probe: libggs vs libggs_probe (GGS_REC_PROBE: 8 consecutive
# visits blend the same record), raster ms and per-wave timing (GGS_TIMING builds).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd
for c in sa2 sa16 512; do
  timeout -k 10 300 python tools/probe/rtime.py --config $c --rounds 2 $P/libggs.so $P/libggs_probe.so > gpurun_out/recp_$c.log 2>&1 || exit $?
  grep SUMMARY gpurun_out/recp_$c.log
done
for L in libggs_timing libggs_tprobe; do
  for cfg in "--size 2048 --splats 4096 --batch 1" "--size 512 --splats 256 --batch 128"; do
    echo "== $L $cfg"; GGS_LIB=$PWD/$P/$L.so timeout -k 10 120 python tools/probe/wave_timing_cfg.py $cfg | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k: d[k] for k in ('span_us','wave_us','phase_frac','blended','clk_per_blended_visit_p50','mean_live')})" || exit $?
  done
done
