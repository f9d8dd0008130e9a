#!/bin/bash
# concat-free ASPP / decoder: kernel + model tests, then the DeepLab preset bench with and without
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_train_gpu.py \
  -k "channel_slice or concat_free or deeplab_preset" > gpurun_out/concat_tests.log 2>&1
for cf in 0 1; do
  TDL_CONCAT_FREE=$cf timeout -k 10 200 python bench.py --model deeplab_ref --steps 30 --warmup 10 \
    > gpurun_out/concat_bench_$cf.log 2>&1
  tail -1 gpurun_out/concat_bench_$cf.log
done
