# round 3: folded-BN inference path — GPU tests, then inference bench A/B (folded vs unfolded, eager vs graph)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_inference.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_infer.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "folded~|passed|failed|Error" gpurun_out/pytest_infer.log | tail -12
[ $rc -eq 0 ] || exit $rc
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 python bench.py --mode infer "$@" > gpurun_out/inf_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/inf_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/inf_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run r50_b1024_fold --steps 20 --warmup 5
run r50_b1024_nofold --steps 20 --warmup 5 --no-fold
run r50_b1024_fold_graph --steps 20 --warmup 5 --graph
run r50_b32_fold --batch 32 --steps 50 --warmup 10
run r50_b32_fold_graph --batch 32 --steps 50 --warmup 10 --graph
run r50_b32_nofold_graph --batch 32 --steps 50 --warmup 10 --graph --no-fold
run r50_b1_fold_graph --batch 1 --steps 100 --warmup 10 --graph
run r152_b1024_fold --model resnet152 --steps 10 --warmup 3
run xc_b256_fold --model xception41 --image-size 299 --batch 256 --steps 10 --warmup 3
run xc_b256_nofold --model xception41 --image-size 299 --batch 256 --steps 10 --warmup 3 --no-fold
echo done
