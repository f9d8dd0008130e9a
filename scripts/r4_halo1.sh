#!/bin/bash
# round 4: halo conv numerics, then same-box A/B vs the implicit-GEMM selection, then bench
bash scripts/gpu_run.sh \
  "halo_tests:400:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'halo or conv_fwd_dgrad_wgrad or dgrad_bnstat or dgrad_relu_mask or dgrad_accumulate' -p no:cacheprovider" \
  "halo_ab:300:python -u bench/halo_ab.py --batch 1024 --out gpurun_out/halo_ab.json" \
  "bench_r50:300:python -u bench.py"
