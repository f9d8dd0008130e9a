# round 3 (end): full GPU suite + smoke on the final build, then the README's bench rows
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_final3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_final3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke3.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/smoke3.log; exit 1; }
tail -1 gpurun_out/smoke3.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 python bench.py "$@" > gpurun_out/fin_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/fin_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/fin_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run r50a --steps 20 --warmup 5
run r50b --steps 20 --warmup 5
run xc --model xception41 --image-size 299 --batch 128 --steps 20 --warmup 5
run dl64 --model deeplab_ref --steps 40 --warmup 5
run dl64g --model deeplab_ref --steps 40 --warmup 5 --graph
run dl32g --model deeplab_ref --batch 32 --steps 40 --warmup 5 --graph
run dl64f32 --model deeplab_ref --dtype fp32 --steps 30 --warmup 5
run r152f8g --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5
run inf_r50 --mode infer --steps 20 --warmup 5
run inf_dl --mode infer --model deeplab_ref --batch 64 --steps 50 --warmup 10 --graph
run inf_dl_nofold --mode infer --model deeplab_ref --batch 64 --steps 50 --warmup 10 --graph --no-fold
echo done
