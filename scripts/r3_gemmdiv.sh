# round 3: register-staged conv kernel with magic-number divisions in its load loop — kernel tests + same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q --timeout 250 --timeout-method thread -k "conv or gemm or wgrad or oracle or side_stream" > gpurun_out/pytest_gemmdiv.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gemmdiv.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/wgrad_ab.py --batch 1024 --rounds 2 --variants default --shapes "56,64,64,3,1,1;28,128,128,3,1,1;14,256,256,3,1,1" > gpurun_out/gd_wgrad_new.log 2>&1 || exit 1
TDL_EXT_SO=ab/_C_f8l.so timeout -k 10 300 python tools/wgrad_ab.py --batch 1024 --rounds 2 --variants default --shapes "56,64,64,3,1,1;28,128,128,3,1,1;14,256,256,3,1,1" > gpurun_out/gd_wgrad_old.log 2>&1 || exit 1
echo old; grep -v amdgpu gpurun_out/gd_wgrad_old.log; echo new; grep -v amdgpu gpurun_out/gd_wgrad_new.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/gd_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/gd_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/gd_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run old0 TDL_EXT_SO=ab/_C_f8l.so
run new0 TDL_X=0
run old1 TDL_EXT_SO=ab/_C_f8l.so
run new1 TDL_X=0
echo done
