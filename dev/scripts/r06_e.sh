R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_train_gpu.py -k "large_batch" tests/test_kernels_gpu.py -k "bn_relu_max_pool or large_batch" > gpurun_out/r06_e.log 2>&1
echo "rc=$?"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_e.log | tail -5
