#!/bin/bash
# full GPU test suite (the driver's round-end tier) on the current build
bash scripts/gpu_run.sh \
  "gpu_suite:1100:python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider"
