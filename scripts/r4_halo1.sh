#!/bin/bash
# round 4: halo conv numerics, same-box A/B vs the implicit-GEMM selection, bench off/on, new tests
bash scripts/gpu_run.sh \
  "halo_tests:400:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'halo or conv_fwd_dgrad_wgrad or dgrad_bnstat or dgrad_relu_mask or dgrad_accumulate or lovasz' -p no:cacheprovider" \
  "halo_ab:300:python -u bench/halo_ab.py --batch 1024 --out gpurun_out/halo_ab.json" \
  "bench_r50:240:python -u bench.py" \
  "bench_r50_halo:240:TDL_HALO=1 python -u bench.py" \
  "tests_new:700:python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_model_classifier.py tests/test_train_gpu.py -k 'deterministic or fp8_graph or classifier or async_saver or graph_training' -m gpu -p no:cacheprovider"
