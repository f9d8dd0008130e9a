# round 3: ResNet-50 b1024 bench under kernel-routing knobs (same box, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/knob_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/knob_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/knob_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run base0 TDL_X=0
run glds2 TDL_CONV_GLDS=2
run base1 TDL_X=0
run glds2b TDL_CONV_GLDS=2
echo done
