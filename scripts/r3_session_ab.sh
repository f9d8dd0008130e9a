# round 3: session-start build (ab/_C_24e082f.so) vs the final build on the other models (same box, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # name, so, args...
  local n=$1; local so=$2; shift 2
  env TDL_EXT_SO=$so timeout -k 10 240 python bench.py "$@" > gpurun_out/sab_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/sab_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/sab_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
NEW=$(ls tensorflowdistributedlearning_amd/_C*.so)
OLD=ab/_C_24e082f.so
DL="--model deeplab_ref --steps 40 --warmup 5 --graph"
run dl_old0 $OLD $DL
run dl_new0 $NEW $DL
run dl_old1 $OLD $DL
run dl_new1 $NEW $DL
XC="--model xception41 --image-size 299 --batch 128 --steps 20 --warmup 5"
run xc_old $OLD $XC
run xc_new $NEW $XC
R5="--steps 20 --warmup 5"
run r50_old $OLD $R5
run r50_new $NEW $R5
echo done
