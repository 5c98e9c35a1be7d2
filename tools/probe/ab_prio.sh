set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=genetic-gaussian-splats_amd
timeout -k 10 400 python tools/probe/rtime.py --config ga24 --rounds 3 $P/libggs_base.so $P/libggs_prio.so 2>&1 | grep SUMMARY || exit 1
timeout -k 10 400 python tools/probe/rtime.py --config 512 --rounds 3 $P/libggs_base.so $P/libggs_prio.so 2>&1 | grep SUMMARY || exit 1
timeout -k 10 400 python tools/probe/rtime.py --config sa2 --rounds 3 $P/libggs_base.so $P/libggs_prio.so 2>&1 | grep SUMMARY || exit 1
for i in 1 2; do for L in base prio; do
  GGS_LIB=$PWD/$P/libggs_$L.so timeout -k 10 200 python3 tools/bench_ga.py --preset default --backend device --gens 4000 --profile-gens 0 > gpurun_out/ga_$L.$i.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ga_$L.$i.json')); print('$L GA', d['value'], d['best_fit'])"
done; done
