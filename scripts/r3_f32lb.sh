# round 3: fp32 conv launch bounds (register allocation) — tests + preset bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_f32_gpu.py -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_f32.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_f32.log
[ $rc -ge 124 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --model deeplab_ref --dtype fp32 --steps 30 --warmup 5 > gpurun_out/dlf32_lb$i.log 2>&1 || exit $?
  echo "lb run $i $(tail -1 gpurun_out/dlf32_lb$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python bench.py --model deeplab_ref --dtype fp32 --batch 32 --steps 30 --warmup 5 > gpurun_out/dlf32_lb_b32.log 2>&1 || exit $?
echo "b32 $(tail -1 gpurun_out/dlf32_lb_b32.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
echo done
