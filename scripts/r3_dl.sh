#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_train_gpu.py \
  -k "dadd or fused_residual or deeplab_preset or concat_free" > gpurun_out/dl_tests.log 2>&1
tail -2 gpurun_out/dl_tests.log
for a in "" "--batch 32 --graph"; do
  for v in 1 0; do
    TDL_DL_FUSE_RES=$v timeout -k 10 300 python bench.py --model deeplab_ref $a --steps 40 --warmup 5 > gpurun_out/dl_bench.log 2>&1
    echo "fuse=$v $a $(tail -1 gpurun_out/dl_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dl3 -o dl -- \
  python bench.py --model deeplab_ref --steps 10 --warmup 3 > gpurun_out/prof_dl3.log 2>&1
echo done
