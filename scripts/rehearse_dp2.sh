# Two ranks sharing the one GPU of a gpurun box: the multi-rank bench path (rendezvous, bucketed
# async all-reduce overlapped with backward, barrier-bracketed timing, MAX over ranks) with gloo.
R=$GRAFT_REPO_ROOT
export TDL_SHARE_GPU=1 MASTER_ADDR=127.0.0.1
TDL_DIST_BACKEND=gloo timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 $R/bench.py --gpus 2 --steps 3 --warmup 1 --batch 32 \
  > $R/gpurun_out/dp2_gloo.log 2>&1 || exit $?
# (RCCL itself refuses two ranks on one device: "Duplicate GPU detected"; the 8-GPU node runs it)
