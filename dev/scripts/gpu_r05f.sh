bash scripts/gpu_run.sh \
 "t_fp8:900:python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_kernels_gpu.py tests/test_bucket_order_gpu.py -k fp8 -p no:cacheprovider"
