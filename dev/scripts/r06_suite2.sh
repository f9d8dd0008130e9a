R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  --ignore=tests/test_kernels_gpu.py --ignore=tests/test_conv_route_gpu.py --ignore=tests/test_f32_gpu.py tests > gpurun_out/r06_suite2.log 2>&1
echo "suite2 rc=$?"; grep -E "FAILED|ERROR" gpurun_out/r06_suite2.log | head -20; tail -2 gpurun_out/r06_suite2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/r06_smoke.log
