bash scripts/gpu_run.sh \
 "t_order:900:python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_bucket_order_gpu.py -p no:cacheprovider" \
 "t_misc:600:python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_bnconv.py tests/test_kernels_gpu.py -k 'resnet50_step or softmax_eval' -m gpu -p no:cacheprovider" \
 "t_det:600:python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_train_gpu.py -k deterministic -p no:cacheprovider" \
 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'"
