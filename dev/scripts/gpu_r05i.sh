bash scripts/gpu_run.sh \
 "t_flip:600:python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py -k 'flat_flips or graph or deterministic' tests/test_kernels_gpu.py -k 'dgrad_as_forward or flat_flips or graph or deterministic' -p no:cacheprovider" \
 "bench:300:python bench.py" \
 "bench2:300:python bench.py"
