# depthwise tile height sweep at the Xception-41 b128 shapes (per-process knob TDL_DW_TR), then
# the Xception bench at the two best settings
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for tr in 32 12 10 7; do
  echo "== TDL_DW_TR=$tr"
  TDL_DW_TR=$tr timeout -k 10 200 python dev/tools/dw_micro.py 2>&1 | grep -v amdgpu || exit $?
done
for tr in 32 10 32 10; do
TDL_DW_TR=$tr timeout -k 10 300 python bench.py --model xception41 --batch 128 --image-size 299 > gpurun_out/r06_x_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_x_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('xception41 b128 TDL_DW_TR=$tr', d['value'], d['ms_per_step'])"
done
