#!/bin/bash
# One GPU session after a change: parity tests, smoke, bench (N=1 plain and
# under torchrun at world 1), then the rocprofv3 passes of tools/profile.sh.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 1 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/bench_torchrun.log 2>&1 || exit $?
grep metric gpurun_out/bench_torchrun.log | cut -c1-300
[ -n "${PROFILE_TAG:-}" ] && bash tools/profile.sh "$PROFILE_TAG"
exit 0
