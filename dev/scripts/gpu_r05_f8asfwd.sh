# fp8 dgrad as the forward conv: kernel + route tests, then the ResNet-152 fp8 graph A/B of
# TDL_FP8_DGRAD_AS_FWD=1 (1x1 stride-1 convs, default) vs 2 (every stride-1 conv) vs 0 (off)
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_conv_route_gpu.py -k "fp8_as_forward or route" > gpurun_out/fa_tests.log 2>&1
: > gpurun_out/fa_ab.log
run() { env TDL_FP8_DGRAD_AS_FWD=$1 timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o '"value": [0-9.]*' | sed "s/^/mode$1 /" >> gpurun_out/fa_ab.log; }
for i in 1 2; do run 1; run 2; run 0; done
