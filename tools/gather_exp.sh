#!/bin/bash
# A/B of the per-batch fitness all-gather in bench.py at world 1 under torchrun
# (GGS_BENCH_GATHER modes), plus the plain N=1 run for reference.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for g in ${MODES:-none rccl rccl-overlap torch torch-sync}; do
  GGS_BENCH_GATHER=$g timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 500 --warmup 10 \
      --no-cpu-baseline > gpurun_out/bench_tr_$g.log 2>&1
done
timeout -k 10 200 python bench.py --steps 500 --warmup 10 --no-cpu-baseline > gpurun_out/bench_plain.log 2>&1
