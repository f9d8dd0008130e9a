bash scripts/gpu_run.sh \
 "t_fp8:900:python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_kernels_gpu.py tests/test_bucket_order_gpu.py -k fp8 -p no:cacheprovider" \
 "sweep:600:python dev/tools/fp8_policy_sweep.py --repeat 2 --variants bf16,default" \
 "r152_bf16:400:python bench.py --model resnet152 --batch 256 --graph" \
 "r152_fp8:400:python bench.py --model resnet152 --batch 256 --graph --fp8" \
 "r152_fp8b:400:python bench.py --model resnet152 --batch 256 --graph --fp8" \
 "stem:300:python dev/tools/stem_ab.py"
