#!/bin/bash
# round 4: halo fwd/dgrad/wgrad numerics + A/B, serial-step kernel profile, fixed new tests
R=$GRAFT_REPO_ROOT
bash scripts/gpu_run.sh \
  "halo_tests:400:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'halo' -p no:cacheprovider" \
  "halo_ab:400:python -u bench/halo_ab.py --batch 1024 --out gpurun_out/halo_ab.json" \
  "prof_serial:300:cd /tmp && TMPDIR=/tmp TDL_WGRAD_STREAM=0 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_serial -o run -- python3 $R/bench.py --steps 5 --warmup 3" \
  "prof_conc:300:cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_conc -o run -- python3 $R/bench.py --steps 5 --warmup 3" \
  "tests_new:700:python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_model_classifier.py tests/test_train_gpu.py -k 'deterministic or classifier or async_saver or graph_training' -m gpu -p no:cacheprovider"
