# round 3: ds_read immediate offsets for the KC fragment reads — kernel tests + same-box bench A/B vs the fast-loop build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "conv or glds or dgrad or wgrad or fp8" > gpurun_out/pytest_ldsimm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ldsimm.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/li_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/li_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/li_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run fl0 TDL_EXT_SO=ab/_C_fl.so
run imm0 TDL_X=0
run fl1 TDL_EXT_SO=ab/_C_fl.so
run imm1 TDL_X=0
echo done
