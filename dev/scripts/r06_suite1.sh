R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py tests/test_conv_route_gpu.py tests/test_f32_gpu.py > gpurun_out/r06_suite1.log 2>&1
echo "suite1 rc=$?"; grep -E "FAILED|ERROR" gpurun_out/r06_suite1.log | head -20; tail -2 gpurun_out/r06_suite1.log
