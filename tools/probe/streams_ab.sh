#!/bin/bash
# bench.py at 4 and 8 HIP streams (streams must divide bench.RING = 8) and 8 / 16
# hardware queues, alternated (2 rounds)
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --streams 4 > gpurun_out/st_4q8.$i.log 2>&1
  GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --streams 4 > gpurun_out/st_4q16.$i.log 2>&1
  GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --streams 8 > gpurun_out/st_8q16.$i.log 2>&1
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --streams 8 > gpurun_out/st_8q8.$i.log 2>&1
done
