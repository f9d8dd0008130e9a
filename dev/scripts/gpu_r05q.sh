bash scripts/gpu_run.sh \
 "t_route:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_route_gpu.py tests/test_kernels_gpu.py -k 'route or stem' -p no:cacheprovider" \
 "b_on:300:python bench.py" \
 "b_off:300:TDL_ROUTE_OFF=fwd.glds.stem python bench.py" \
 "b_on2:300:python bench.py" \
 "b_off2:300:TDL_ROUTE_OFF=fwd.glds.stem python bench.py"
