# round 3 (late): 32x32x16 MFMA K loop (TDL_M32=1) re-measured after the VALU cuts — same box, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/m32b_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/m32b_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/m32b_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run base0 TDL_X=0
run m32_0 TDL_M32=1
run base1 TDL_X=0
run m32_1 TDL_M32=1
echo done
