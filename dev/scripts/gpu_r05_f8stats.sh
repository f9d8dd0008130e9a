# fp8 dgrad with fused BN-backward statistics: kernel + fp8 training tests, then the ResNet-152
# fp8 graph A/B against TDL_FP8_DGRAD_STATS=0 (the BN reduce pass), and bf16 on the same box
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "fp8" tests/test_train_gpu.py tests/test_conv_route_gpu.py > gpurun_out/f8s_tests.log 2>&1
: > gpurun_out/f8s_ab.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/fused /' >> gpurun_out/f8s_ab.log
  TDL_FP8_DGRAD_STATS=0 timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/reduce /' >> gpurun_out/f8s_ab.log
done
timeout -k 10 300 python bench.py --model resnet152 --batch 256 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/bf16 /' >> gpurun_out/f8s_ab.log
