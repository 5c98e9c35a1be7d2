#!/bin/bash
# World-1 proxy for N>1: bench under torchrun with the single-rank gather routed
# through RCCL (GGS_COMM_RCCL_SELF=1) vs the copy kernel, 2 streams vs 1.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
trun() { timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
         --master-port 29511 bench.py --gpus 1 --no-cpu-baseline "$@"; }
for rep in 1 2; do
  GGS_COMM_RCCL_SELF=1 trun > gpurun_out/trr.log 2>&1; grep -o '"value": [0-9.]*\|"value_one_stream": [0-9.]*' gpurun_out/trr.log | tr '\n' ' ' | sed 's/^/rccl-self 2 streams: /'; echo
  trun > gpurun_out/trc.log 2>&1; grep -o '"value": [0-9.]*\|"value_one_stream": [0-9.]*' gpurun_out/trc.log | tr '\n' ' ' | sed 's/^/copy 2 streams: /'; echo
done
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/plain.log 2>&1; grep -o '"value": [0-9.]*\|"value_one_stream": [0-9.]*' gpurun_out/plain.log | tr '\n' ' ' | sed 's/^/plain: /'; echo
