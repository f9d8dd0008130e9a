"""One rank of the data-parallel equality test (tests/test_train_gpu.py::
test_two_ranks_equal_single_process_average), started by torch.distributed.run.

Every rank builds the same ResNet-50 (seed 1234, then the rank-0 broadcast of Trainer), trains
``steps`` SGD-momentum steps on its own synthetic half-batch (``imagenet_batch(seed=rank)``) in
deterministic mode (csrc/kernels/det.hip: fixed-order reductions, so a rank's gradients are a
pure function of its weights and data), with the weight gradients on the side stream and the
gradients averaged by the bucketed all-reduce (``grad_dtype`` fp32 or bf16 buckets), and writes
its fp32 master weights and losses to ``OUT/rank{r}.pt``.

  python -m torch.distributed.run --nproc-per-node 2 ... tests/_dp_worker.py OUT fp32 3
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# the shape every rank trains on (the test's single-process reference reads these)
BATCH, SIZE, LR, MOMENTUM, WD = 4, 64, 0.05, 0.9, 1e-4


def main():
    out_dir, grad_dtype, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    import torch
    from tensorflowdistributedlearning_amd import models
    from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch
    from tensorflowdistributedlearning_amd.engine.trainer import Trainer
    from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy, streams
    from tensorflowdistributedlearning_amd.ops.common import ext
    from tensorflowdistributedlearning_amd.parallel.dist import init_distributed, shutdown
    ctx = init_distributed()
    assert ctx.world_size == 2 and ctx.device.type == "cuda", (ctx.world_size, ctx.device)
    ext().det_set(1)
    torch.manual_seed(1234)
    model = models.build("resnet50", num_classes=1000)
    tr = Trainer(model, softmax_cross_entropy, ctx.device, "sgd",
                 dict(lr=LR, momentum=MOMENTUM, weight_decay=WD), ctx=ctx,
                 grad_comm_dtype=torch.bfloat16 if grad_dtype == "bf16" else torch.float32)
    x, y = imagenet_batch(BATCH, SIZE, device=ctx.device, seed=ctx.rank)
    losses = [tr.train_step(x, y)[0] for _ in range(steps)]
    torch.cuda.synchronize(ctx.device)
    torch.save({"master": tr.flat.master.detach().cpu(),
                "losses": [float(v) for v in losses],
                "side_stream": streams.enabled(),
                "buckets": len(tr.bucketer.buckets),
                "early": tr.bucketer.early_launches},
               os.path.join(out_dir, f"rank{ctx.rank}.pt"))
    ctx.barrier()
    shutdown()


if __name__ == "__main__":
    main()
