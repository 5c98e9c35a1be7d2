#!/bin/bash
# round 6: parity of the visit-word raster + host pipeline, then A/Bs vs HEAD's build (libggs_base)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host_errors.py tests/test_degenerate_splats.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t3.log 2>&1
rc=$?; tail -3 gpurun_out/t3.log; [ $rc -eq 0 ] || exit $rc
ALT="libggs_base libggs" CFGS="512 ga24 sa2 1024" ROUNDS=3 bash tools/probe/ab_rtime.sh || exit 1
# SA round width at the start of a configs[4] run: adaptive (0) vs fixed 1 / 2 / 3
for w in 0 1 2 3; do
  timeout -k 10 300 python3 tools/bench_sa.py --only device_loop_full --repeat 3 --speculate $w > gpurun_out/sa_width_$w.json 2>&1 || { tail -3 gpurun_out/sa_width_$w.json; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['device_loop_full']; print('width', sys.argv[2], d['iters_per_s'], d['runs_iters_per_s'], 'rounds', d['launches'], 'evaluated', d['evaluated'], 'us/round', d['us_per_round'])" gpurun_out/sa_width_$w.json $w
done
# the headline's stream count: 2 / 4 / 8 independent batches in flight
for s in 4 8 2 4 8; do
  timeout -k 10 300 python3 bench.py --streams $s --no-cpu-baseline --extras 0 > gpurun_out/bench_streams_$s.log 2>&1 || { tail -3 gpurun_out/bench_streams_$s.log; exit 1; }
  grep '^{' gpurun_out/bench_streams_$s.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams', $s, d['value'], d['ms_per_step'])"
done
