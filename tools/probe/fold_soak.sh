set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 0 1; do
  GGS_UNFUSED_FINALIZE=$v SOAK_GENS=100000 timeout -k 10 200 python tools/probe/fold_soak.py > gpurun_out/soak_default_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/soak_default_$v.log
  GGS_UNFUSED_FINALIZE=$v SOAK_SHAPE=bench SOAK_GENS=20000 timeout -k 10 200 python tools/probe/fold_soak.py > gpurun_out/soak_bench_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/soak_bench_$v.log
done
