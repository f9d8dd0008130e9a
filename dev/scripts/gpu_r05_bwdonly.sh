# e5m2-only BN input gradients (fp8_bwd_only): equivalence test + fp8 tests, then the ResNet-152
# fp8 graph A/B (TDL_FP8_BWD_ONLY=0 switches the flag off in models.enable_fp8)
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_train_gpu.py -k "fp8_bwd_only" > gpurun_out/bo_tests.log 2>&1
: > gpurun_out/bo_ab.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/only /' >> gpurun_out/bo_ab.log
  TDL_FP8_BWD_ONLY=0 timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/both /' >> gpurun_out/bo_ab.log
done
timeout -k 10 300 python bench.py --model resnet152 --batch 256 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/bf16 /' >> gpurun_out/bo_ab.log
