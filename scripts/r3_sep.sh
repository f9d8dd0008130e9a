#!/bin/bash
# separable-path BN statistics fusion: kernel + model tests, Xception / DeepLab / ResNet-50 benches
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_train_gpu.py \
  -k "depthwise or bnstat or xception or deeplab or premasked or fused_bn" > gpurun_out/sep_tests.log 2>&1
tail -3 gpurun_out/sep_tests.log
for m in "xception41 --image-size 299 --batch 128" "deeplab_ref --batch 32 --graph" "resnet50"; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/sep_bench.log 2>&1
  tail -1 gpurun_out/sep_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], d["value"], d["ms_per_step"])'
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_xc2 -o xc -- \
  python bench.py --model xception41 --image-size 299 --batch 64 --steps 5 --warmup 2 > gpurun_out/prof_xc2.log 2>&1
echo done
