#!/bin/bash
# separable-path BN statistics fusion + DeepLab fused residual units: tests, benches, profiles
set -e
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_train_gpu.py \
  -k "xception_fused or fused_residual or deeplab_bf16" > gpurun_out/sep_tests.log 2>&1
tail -3 gpurun_out/sep_tests.log
for m in "xception41 --image-size 299 --batch 128" "deeplab_ref --batch 32 --graph" "deeplab_ref" "resnet50"; do
  timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 > gpurun_out/sep_bench.log 2>&1
  tail -1 gpurun_out/sep_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], d["config"]["global_batch"], d["value"], d["ms_per_step"])'
done
TDL_DL_FUSE_RES=0 timeout -k 10 300 python bench.py --model deeplab_ref --steps 30 --warmup 5 > gpurun_out/sep_bench.log 2>&1
tail -1 gpurun_out/sep_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("deeplab unfused", d["value"], d["ms_per_step"])'
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_xc2 -o xc -- \
  python bench.py --model xception41 --image-size 299 --batch 64 --steps 5 --warmup 2 > gpurun_out/prof_xc2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dl2 -o dl -- \
  python bench.py --model deeplab_ref --steps 10 --warmup 3 > gpurun_out/prof_dl2.log 2>&1
echo done
