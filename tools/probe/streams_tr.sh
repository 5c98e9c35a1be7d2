#!/bin/bash
# bench.py under torch.distributed.run (world 1, RCCL gathers) at 2 and 4 streams
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2; do
 for s in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 1 --steps 200 --warmup 10 --no-cpu-baseline --streams $s > gpurun_out/tr_$s.$i.log 2>&1
 done
done
