# round 3: MC (transposed) fragment reads with immediate offsets + 1x1 stride-1 weight-gradient DMAs without pixel
# divisions — kernel tests + same-box bench A/B vs the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q --timeout 250 --timeout-method thread -k "conv or glds or dgrad or wgrad or fp8 or oracle or side_stream" > gpurun_out/pytest_mcimm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_mcimm.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/mi_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/mi_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/mi_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run imm0 TDL_EXT_SO=ab/_C_imm.so
run mc0 TDL_X=0
run imm1 TDL_EXT_SO=ab/_C_imm.so
run mc1 TDL_X=0
echo done
