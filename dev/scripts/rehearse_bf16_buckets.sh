# bf16 vs fp32 gradient buckets, ResNet-152, two gloo ranks sharing the box's GPU (the multi-rank
# bench path; RCCL refuses two ranks on one device): standalone_ms / exposed_ms from bench.py
R=$GRAFT_REPO_ROOT
export TDL_SHARE_GPU=1 MASTER_ADDR=127.0.0.1 TDL_DIST_BACKEND=gloo
for dt in fp32 bf16; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29613 $R/bench.py --gpus 2 --steps 3 --warmup 1 \
    --batch 32 --model resnet152 --grad-dtype $dt > $R/gpurun_out/dp2_r152_$dt.log 2>&1 || exit $?
done
