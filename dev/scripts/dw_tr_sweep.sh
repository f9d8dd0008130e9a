# depthwise tile height per shape (dev/tools/dw_micro.py under TDL_DW_TR caps)
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out; : > gpurun_out/dw_tr.log
for tr in 32 16 10 7; do
  echo "== TDL_DW_TR=$tr" >> gpurun_out/dw_tr.log
  TDL_DW_TR=$tr timeout -k 10 120 python dev/tools/dw_micro.py 2>/dev/null | grep -v "^s2 dgrad" >> gpurun_out/dw_tr.log
done
