set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/comm_tests.log 2>&1 || { tail -30 gpurun_out/comm_tests.log; exit 1; }
tail -2 gpurun_out/comm_tests.log
timeout -k 10 300 python tools/bench_ga.py --backend device --gens 200 2>&1 | grep metric
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 tools/bench_ga.py --backend device --gens 200 2>&1 | grep metric
timeout -k 10 300 python tools/bench_ga.py --backend device --gens 5 --size 1024 --splats 1024 --pop 4096 2>&1 | grep metric
