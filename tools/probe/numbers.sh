#!/bin/bash
# The DESIGN section 6 numbers besides the headline: configs[2] and configs[3] at N=1,
# the device GA at the bench size and at configs[3], the SA at configs[4] (start and
# late regime).  Each step under its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
j() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({k: d.get(k) for k in sys.argv[1:]}))" "$@"; }
timeout -k 10 300 python bench.py --config 1024 --steps 10 --warmup 2 --no-cpu-baseline | j value ms_per_step value_one_stream kernels_ms_per_launch || exit $?
timeout -k 10 300 python bench.py --config 1024x8 --steps 5 --warmup 1 --no-cpu-baseline | j value ms_per_step config || exit $?
timeout -k 10 300 python tools/bench_ga.py --backend device --gens 2000 | j value ms_per_gen candidate_renders_per_s || exit $?
timeout -k 10 300 python tools/bench_ga.py --backend device --size 1024 --splats 1024 --pop 4096 --gens 10 | j value ms_per_gen candidate_renders_per_s || exit $?
timeout -k 10 300 python tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 3 | j device_loop_full || exit $?
timeout -k 10 600 python tools/bench_sa.py --only device_loop_full --dev-iters 200 --repeat 3 --warm 2000 --temp0 1e-6 | j device_loop_full || exit $?
