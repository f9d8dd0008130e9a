bash scripts/gpu_run.sh \
 "t_route:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_route_gpu.py -p no:cacheprovider" \
 "t_kern:900:python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_bnconv.py -p no:cacheprovider" \
 "bench:300:python bench.py"
