set -u
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import torch; print(torch.cuda.Stream.priority_range())" > gpurun_out/prio.log 2>&1
for v in 512:4 1024:4 1024:2 2048:2 256:8; do
  b=${v%%:*}; u=${v##*:}
  TDL_BN_RED_BLOCKS=$b TDL_BN_RED_U=$u BN_TAG=b${b}u$u timeout -k 10 120 python tools/bn_micro.py >> gpurun_out/bn_micro.log 2>&1 || exit $?
done
for p in 0 -1 0 -1; do
  TDL_STREAM_PRIO=$p timeout -k 10 120 python bench.py --steps 30 --warmup 5 >> gpurun_out/prio_bench.log 2>&1 || exit $?
done
