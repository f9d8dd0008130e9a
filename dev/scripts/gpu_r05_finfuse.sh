# BN finalize inside the apply launch: full GPU suite, then same-box A/Bs vs TDL_BN_FIN_FUSE=0
# (records an A/B of a reverted change: the TDL_BN_FIN_FUSE knob is not in the tree; profiles/r05_bn_finalize_fuse_ab.txt)
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/ff_suite.log 2>&1
: > gpurun_out/ff_ab.log
for i in 1 2; do
  timeout -k 10 300 python bench.py 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/r50 fused /' >> gpurun_out/ff_ab.log
  TDL_BN_FIN_FUSE=0 timeout -k 10 300 python bench.py 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/r50 sep   /' >> gpurun_out/ff_ab.log
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/f8 fused /' >> gpurun_out/ff_ab.log
  TDL_BN_FIN_FUSE=0 timeout -k 10 300 python bench.py --model resnet152 --batch 256 --fp8 --graph --steps 20 --warmup 5 2>/dev/null | tail -1 | grep -o "\"value\": [0-9.]*" | sed 's/^/f8 sep   /' >> gpurun_out/ff_ab.log
done
