#!/bin/bash
# non-temporal BN streaming A/B on the headline ResNet-50 b1024 bench (alternating rounds)
set -e
mkdir -p gpurun_out
TDL_BN_NT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py -k "bn_" > gpurun_out/ntab_tests.log 2>&1
tail -1 gpurun_out/ntab_tests.log
for rep in 1 2 3; do
  for v in 0 1; do
    TDL_BN_NT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ntab.log 2>&1
    echo "nt=$v $(tail -1 gpurun_out/ntab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
