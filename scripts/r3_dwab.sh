#!/bin/bash
# depthwise fused-statistics A/B on Xception-41 b128 (alternating), then the dw kernel tests
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py -k "depthwise" > gpurun_out/dwab_tests.log 2>&1
tail -1 gpurun_out/dwab_tests.log
run() {
  env "$@" timeout -k 10 300 python bench.py --model xception41 --image-size 299 --batch 128 --steps 20 --warmup 5 > gpurun_out/dwab.log 2>&1
  echo "$* $(tail -1 gpurun_out/dwab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for rep in 1 2; do
  run TDL_DW_STATS=1
  run TDL_DW_STATS=0
  run TDL_DW_STATS=1 TDL_DW_STAT_WG=512
  run TDL_DW_STATS=1 TDL_DW_STAT_WG=8192
  run TDL_BNSTAT_FUSE=0 TDL_DW_STATS=0
done
