"""fp8 dgrad vs bf16 dgrad on identical weights (lr = 0, so both models stay equal): per-layer
cosine of the parameter gradients after the e5m2 scalers warmed up.
  python dev/tools/fp8_dgrad_check.py [--depth 18] [--train-bn]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd import models  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=18)
    ap.add_argument("--fwd-fp8", type=int, default=1)
    ap.add_argument("--frozen", action="store_true")
    a = ap.parse_args()
    gpu = torch.device("cuda")
    torch.manual_seed(0)
    nets = [models.build(f"resnet{a.depth}", num_classes=10) for _ in range(3)]
    for n in nets[1:]:
        n.load_state_dict(nets[0].state_dict())
    if a.fwd_fp8:
        models.enable_fp8(nets[0], dgrad=False)
    models.enable_fp8(nets[1], dgrad=True)
    trs = [Trainer(n, softmax_cross_entropy, gpu, "sgd", dict(lr=0.0, momentum=0.0)) for n in nets]
    for t in trs:
        t.train_mode = not a.frozen
    x, y = imagenet_batch(32, 64, num_classes=10, device=gpu)
    for _ in range(3):
        for t in trs:
            t.train_step(x, y)
    torch.cuda.synchronize()
    cos = torch.nn.functional.cosine_similarity
    print("whole: fp8-dgrad vs bf16-dgrad", cos(trs[0].flat.grad, trs[1].flat.grad, dim=0).item(),
          " bf16 rerun vs bf16(fwd fp8 off)", cos(trs[0].flat.grad, trs[2].flat.grad, dim=0).item())
    for (n, p0), p1 in zip(nets[0].named_parameters(), nets[1].parameters()):
        c = cos(p0.grad.flatten(), p1.grad.flatten(), dim=0).item()
        r = (p1.grad.norm() / (p0.grad.norm() + 1e-30)).item()
        print(f"{n:45s} cos {c:.4f} norm ratio {r:.3f}")


if __name__ == "__main__":
    main()
