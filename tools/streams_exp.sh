#!/bin/bash
# A/B: batches alternating over 1 / 2 HIP streams (GGS_BENCH_STREAMS), plain
# N=1 and under torchrun (world 1), with the HIP hardware-queue count varied.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tr() { timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
         --master-port 29511 bench.py --gpus 1 --steps 500 --warmup 10 --no-cpu-baseline; }
for q in ${QLIST:-4 8 16}; do
  GPU_MAX_HW_QUEUES=$q GGS_BENCH_STREAMS=2 timeout -k 10 200 python bench.py --steps 500 --warmup 10 --no-cpu-baseline > gpurun_out/bench_q$q.log 2>&1
  grep -o '"value": [0-9.]*' gpurun_out/bench_q$q.log | sed "s/^/plain streams=2 hwq=$q /"
  GPU_MAX_HW_QUEUES=$q GGS_BENCH_STREAMS=2 tr > gpurun_out/bench_tr_q$q.log 2>&1
  grep -o '"value": [0-9.]*' gpurun_out/bench_tr_q$q.log | sed "s/^/torchrun streams=2 hwq=$q /"
done
