cd $GRAFT_REPO_ROOT
timeout -k 5 60 ./dev/tools/tr_b8_probe > gpurun_out/tr_b8.log 2>&1 || exit $?
bash scripts/gpu_run.sh \
 "t_w8:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'wgrad_fp8' -p no:cacheprovider" \
 "t_fp8:900:python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_bucket_order_gpu.py -k fp8 -p no:cacheprovider" \
 "t_route:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_route_gpu.py -p no:cacheprovider" \
 "sweep:600:python dev/tools/fp8_policy_sweep.py --repeat 2 --variants bf16,default" \
 "r152_bf16:400:python bench.py --model resnet152 --batch 256 --graph" \
 "r152_fp8:400:python bench.py --model resnet152 --batch 256 --graph --fp8" \
 "r152_fp8nw:400:TDL_FP8_WGRAD=0 python bench.py --model resnet152 --batch 256 --graph --fp8" \
 "strided:300:python bench/dgrad_strided.py"
