set -e
cd $GRAFT_REPO_ROOT
ALT=${ALT:-libggs_new}
timeout -k 10 300 python tools/probe/bitcmp.py genetic-gaussian-splats_amd/libggs.so genetic-gaussian-splats_amd/$ALT.so > gpurun_out/ab_bitcmp.log 2>&1
for i in 1 2 3; do
 for L in libggs $ALT; do
  GGS_LIB=$PWD/genetic-gaussian-splats_amd/$L.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/ab_$L.$i.log 2>&1
 done
done
