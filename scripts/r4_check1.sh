#!/bin/bash
# round-4 first GPU check: baseline bench + new GPU tests (Model classifier graph loop, fp8 interleave)
bash scripts/gpu_run.sh \
  "bench_r50:300:python -u bench.py" \
  "tests_new:600:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_model_classifier.py tests/test_train_gpu.py::test_fp8_graph_replay_interleaved_with_eager_forwards tests/test_train_gpu.py::test_fp8_graph_replay_matches_eager -m gpu -p no:cacheprovider"
