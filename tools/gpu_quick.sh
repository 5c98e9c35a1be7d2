set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "headline or ga_default" > gpurun_out/pt_headline.log 2>&1; rc=$?; tail -5 gpurun_out/pt_headline.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/bench_a.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/bench_tr.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/bench_b.log 2>&1 || exit $?
for f in bench_a bench_tr bench_b; do python -c "
import json,sys
l=[x for x in open('gpurun_out/$f.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$f', d['value'], d['value_one_stream'], d['value_with_readback'], d['roofline']['frac'], d['valu']['frac'], d['roofline']['bound'])"; done
