# round 3 (late): strength-reduced weight-gradient DMA addressing — tests + same-box A/B; M32 K loop re-measured
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q --timeout 250 --timeout-method thread -k "conv or wgrad or glds or oracle or side_stream" > gpurun_out/pytest_wgsr.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_wgsr.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/ws_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ws_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/ws_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run head0 TDL_EXT_SO=ab/_C_head.so
run new0 TDL_X=0
run head1 TDL_EXT_SO=ab/_C_head.so
run new1 TDL_X=0
run m32_0 TDL_M32=1
run m32_1 TDL_M32=1
echo done
