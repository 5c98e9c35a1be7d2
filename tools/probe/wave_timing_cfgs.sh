set -u
cd $GRAFT_REPO_ROOT
export GGS_LIB=$PWD/genetic-gaussian-splats_amd/libggs_timing.so
for cfg in "--size 2048 --splats 4096 --batch 1" "--size 2048 --splats 4096 --batch 3" "--size 2048 --splats 4096 --batch 16" "--size 512 --splats 256 --batch 128" "--size 1024 --splats 1024 --batch 64"; do
  echo "== $cfg"; timeout -k 10 120 python tools/probe/wave_timing_cfg.py $cfg || exit $?
done
