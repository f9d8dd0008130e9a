"""Where does a HIP-graph-captured data-parallel step (native RCCL collectives captured with the
step, world 1 standing in) differ from the eager one?  Runs one eager twin and one captured
trainer from identical state and prints, per parameter, the gradient difference after each
step — a bucket-shaped pattern would point at collective ordering, isolated small differences
at reduction-order noise.

  python tools/dp_graph_debug.py [--side 0|1] [--steps 2]"""
import argparse
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tensorflowdistributedlearning_amd import models  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy, streams  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch  # noqa: E402
from tensorflowdistributedlearning_amd.parallel.rccl import NativeComm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=0)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--lr", type=float, default=0.0)
    ap.add_argument("--values", action="store_true")
    a = ap.parse_args()
    gpu = torch.device("cuda")
    streams.set_enabled(bool(a.side))
    nc = NativeComm(0, 1, gpu)

    def ctx():
        return SimpleNamespace(is_distributed=True, world_size=2, rank=0, is_main=True, native=nc,
                               all_reduce_async=lambda t: nc.all_reduce(t, async_op=True),
                               broadcast_=lambda t, src=0: t, check=lambda: None,
                               barrier=lambda: None)
    torch.manual_seed(11)
    nets = [models.resnet18(num_classes=10) for _ in range(3)]
    for n in nets[1:]:
        n.load_state_dict(nets[0].state_dict())
    tr = [Trainer(n, softmax_cross_entropy, gpu, "sgd", dict(lr=a.lr, momentum=0.0),
                  ctx=ctx(), bucket_mb=1.0, first_bucket_mb=0.25) for n in nets]
    for t in tr:
        t.train_mode = False
    x, y = imagenet_batch(8, 32, num_classes=10, device=gpu)
    tr[2].capture(x, y, warmup=1)
    tr[0].train_step(x, y)
    tr[1].train_step(x, y)
    print("buckets (index, params, bytes):", tr[0].bucketer.describe())
    for s in range(a.steps):
        tr[0].train_step(x, y)
        tr[1].train_step(x, y)
        tr[2].replay()
        torch.cuda.synchronize()
        print(f"step {s}: eager/eager max|dg| {(tr[0].flat.grad - tr[1].flat.grad).abs().max():.3e}"
              f"  eager/graph max|dg| {(tr[0].flat.grad - tr[2].flat.grad).abs().max():.3e}")
        names = dict(tr[0].model.named_parameters())
        for n, p in names.items():
            lo, hi = tr[0].flat.slice_of(p)
            d01 = (tr[0].flat.grad[lo:hi] - tr[1].flat.grad[lo:hi]).abs().max().item()
            d02 = (tr[0].flat.grad[lo:hi] - tr[2].flat.grad[lo:hi]).abs().max().item()
            ref = tr[0].flat.grad[lo:hi].abs().max().item() + 1e-12
            if d02 > 0 or d01 > 0:
                print(f"   {n:45s} [{lo:9d},{hi:9d}) rel eager/eager {d01 / ref:.2e} "
                      f"eager/graph {d02 / ref:.2e}  max|g| {ref:.3e}")
                if a.values:
                    print("      eager", tr[0].flat.grad[lo:lo + 8].tolist())
                    print("      graph", tr[2].flat.grad[lo:lo + 8].tolist())
        gn = dict(tr[0].model.named_parameters())
        for key in ("stem.bn.beta", "stem.conv.weight"):
            lo, hi = tr[0].flat.slice_of(gn[key])
            print(f"   {key}: max|g| {tr[0].flat.grad[lo:hi].abs().max().item():.3e}")
    nc.synchronize()


if __name__ == "__main__":
    main()
