# fp8 dgrad statistics for residual joins too: kernel + fp8 tests, route tests, then the
# ResNet-152 fp8 graph A/B against TDL_FP8_JOIN_STATS=0
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_conv_route_gpu.py tests/test_bucket_order_gpu.py -k "fp8 or dgrad or bucket" > gpurun_out/fj_tests.log 2>&1
: > gpurun_out/fj_ab.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/join-fused /' >> gpurun_out/fj_ab.log
  TDL_FP8_JOIN_STATS=0 timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/join-reduce /' >> gpurun_out/fj_ab.log
done
