# round 3: predict on the GPU with folded BN + bf16 weight copies; DeepLab preset inference bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_cpu.py tests/test_inference.py -x -v --timeout 200 --timeout-method thread -k "gpu or predict" > gpurun_out/pytest_infer2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_infer2.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 python bench.py --mode infer "$@" > gpurun_out/inf_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/inf_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/inf_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run dl_b64_fold --model deeplab_ref --batch 64 --steps 50 --warmup 10
run dl_b64_nofold --model deeplab_ref --batch 64 --steps 50 --warmup 10 --no-fold
run dl_b64_fold_graph --model deeplab_ref --batch 64 --steps 50 --warmup 10 --graph
run dl_b64_nofold_graph --model deeplab_ref --batch 64 --steps 50 --warmup 10 --graph --no-fold
run dl_b1024_fold --model deeplab_ref --batch 1024 --steps 20 --warmup 5
run dl_b1024_nofold --model deeplab_ref --batch 1024 --steps 20 --warmup 5 --no-fold
run dl_b64_fp32_fold_graph --model deeplab_ref --batch 64 --steps 30 --warmup 5 --graph --dtype fp32
echo done
