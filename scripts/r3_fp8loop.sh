# round 3: fp8 LDS-DMA loop split into the in-tile fast loop — fp8 tests + ResNet-152 fp8 bench A/B vs the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q --timeout 300 --timeout-method thread -k "fp8" > gpurun_out/pytest_fp8loop.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_fp8loop.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 > gpurun_out/f8_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/f8_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/f8_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run mc0 TDL_EXT_SO=ab/_C_mc.so
run f8l0 TDL_X=0
run mc1 TDL_EXT_SO=ab/_C_mc.so
run f8l1 TDL_X=0
echo done
