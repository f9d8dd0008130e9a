# round 3: register-staged dgrad with magic-number divisions — tests + DeepLab preset / ResNet-50 same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_f32_gpu.py -x -q --timeout 250 --timeout-method thread -k "conv or gemm or dgrad or oracle or deeplab" > gpurun_out/pytest_gemmdiv2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gemmdiv2.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py $ARGS > gpurun_out/gd2_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/gd2_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/gd2_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
export ARGS="--model deeplab_ref --steps 40 --warmup 5"
run dl_old0 TDL_EXT_SO=ab/_C_gd.so
run dl_new0 TDL_X=0
run dl_old1 TDL_EXT_SO=ab/_C_gd.so
run dl_new1 TDL_X=0
export ARGS="--steps 20 --warmup 5"
run r50_old TDL_EXT_SO=ab/_C_gd.so
run r50_new TDL_X=0
echo done
