# round 3 (late): full GPU suite + smoke on this build, then register-staged dgrad fastdiv A/B (DeepLab preset, ResNet-50)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_final2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_final2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke2.log; exit 1; }
tail -1 gpurun_out/smoke2.log
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
timeout -k 10 240 python bench.py > gpurun_out/bench_final2.log 2>&1 && tail -1 gpurun_out/bench_final2.log
echo done
