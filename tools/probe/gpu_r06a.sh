set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lpt.py tests/test_gpu_host_errors.py "tests/test_gpu_ga.py::test_device_ga_fused_breed_equals_unfused" "tests/test_gpu_ga.py::test_device_ga_matches_host_ga_with_same_draws" tests/test_gpu_comm.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?; tail -4 gpurun_out/t1.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for L in 1 0; do GGS_PROBE=1 GGS_LIB=$PWD/genetic-gaussian-splats_amd/libggs_probe.so GGS_GA_LPT=$L timeout -k 10 120 python3 tools/probe/lpt_waves.py > gpurun_out/lpt_waves_$L.json 2>&1 || { tail -5 gpurun_out/lpt_waves_$L.json; exit 1; }; cut -c1-1200 gpurun_out/lpt_waves_$L.json; echo; done
