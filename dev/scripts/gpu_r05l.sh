bash scripts/gpu_run.sh \
 "t_asf:900:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'dgrad_as_forward or conv_dgrad or relu_mask or bnstat' -p no:cacheprovider" \
 "t_route:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_route_gpu.py -p no:cacheprovider" \
 "t_train:900:python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py -k 'premasked or join or graph or deterministic or flat_flips' -p no:cacheprovider" \
 "route_r50:300:python tools/route_report.py --model resnet50 --batch 1024" \
 "bench:300:python bench.py" \
 "bench_off:300:TDL_ROUTE_OFF=dgrad.asfwd.strided,dgrad.asfwd.strided.n64 python bench.py" \
 "bench2:300:python bench.py"
