bash scripts/gpu_run.sh \
 "t_asfwd:600:python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k 'dgrad_as_forward or conv_dgrad' -p no:cacheprovider" \
 "dgrad_paths:300:python bench/dgrad_paths.py" \
 "bench_on:300:python bench.py" \
 "bench_off:300:TDL_DGRAD_AS_FWD=0 python bench.py" \
 "bench_on2:300:python bench.py"
