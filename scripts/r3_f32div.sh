# round 3: full GPU suite + fp32 scalar K-step / magic-division change (preset fp32 A/B vs previous numbers)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/pytest_all.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_all.log
[ $rc -ge 124 ] && exit $rc
for b in 64 32; do
  timeout -k 10 300 python bench.py --model deeplab_ref --dtype fp32 --batch $b --steps 30 > gpurun_out/dlf32_div_$b.log 2>&1 || exit $?
  echo "fp32 b$b $(tail -1 gpurun_out/dlf32_div_$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
echo done
