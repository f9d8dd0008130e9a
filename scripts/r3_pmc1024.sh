# round 3: full GPU test suite, then the per-kernel PMC summary of the ResNet-50 b1024 bench step
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_run.sh \
  "pytest:900:python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread" \
  "pmc:600:bash scripts/pmc_bench.sh resnet50 1024 224" \
  "pmcsum:120:python3 tools/pmc_summary.py gpurun_out/pmc_resnet50_sq gpurun_out/pmc_resnet50_fetch gpurun_out/pmc_resnet50_write > gpurun_out/pmc_resnet50_b1024_summary.txt"
