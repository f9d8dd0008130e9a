# round 3: reference preset bf16 at b64 eager vs HIP graph (launch-bound check), fp32 graph b32
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for a in "" "--graph" "" "--graph"; do
  timeout -k 10 300 python bench.py --model deeplab_ref --steps 40 $a > gpurun_out/dlg.log 2>&1 || exit $?
  echo "bf16 b64 $a $(tail -1 gpurun_out/dlg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python bench.py --model deeplab_ref --dtype fp32 --batch 32 --graph --steps 30 > gpurun_out/dlg.log 2>&1 || exit $?
echo "fp32 b32 graph $(tail -1 gpurun_out/dlg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
echo done
