"""How far the bf16 GPU training step sits from the CPU fp32 oracle on the smoke's ResNet-50
(identical bf16-rounded weights and input, plain SGD at lr 1e-3), by batch and image size: the
BN batch statistics of the last stage are taken over batch·(size/32)² values per channel, and few
values amplify the bf16 rounding of the activations.  Prints the per-step losses of both, the
relative gap, and the first step's logit cosine.  Fed the choice of the smoke's shape
(__graft_entry__.smoke, profiles/r06_smoke_oracle_gap.txt)."""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd import _native, models  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch  # noqa: E402

import argparse  # noqa: E402
ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="4x64,8x64,8x96,16x96,8x128,16x128", help="batch x size list")
ap.add_argument("--lr", type=float, default=1e-3)
ap.add_argument("--repeat", type=int, default=1)
args = ap.parse_args()
_native.load()
gpu = torch.device("cuda", 0)
cfgs = [tuple(int(v) for v in c.split("x")) for c in args.configs.split(",")] * args.repeat
for batch, size in cfgs:
    torch.manual_seed(0)
    mc = models.resnet50(num_classes=1000)
    mg = models.resnet50(num_classes=1000)
    mg.load_state_dict(mc.state_dict())
    opt = dict(lr=args.lr, momentum=0.0, weight_decay=0.0)
    tc = Trainer(mc, softmax_cross_entropy, "cpu", "sgd", opt, lowp_dtype=None)
    with torch.no_grad():
        tc.flat.master.copy_(tc.flat.master.bfloat16().float())
        tc.flat.sync_lowp()
    tg = Trainer(mg, softmax_cross_entropy, gpu, "sgd", opt)
    with torch.no_grad():
        tg.flat.master.copy_(tc.flat.master.to(gpu))
        tg.flat.sync_lowp()
    x, y = imagenet_batch(batch, size, device="cpu", dtype=torch.float32)
    x = x.bfloat16().float()
    lc, lg = [], []
    for i in range(4):
        l1, o1 = tc.train_step(x, y)
        l2, o2 = tg.train_step(x.to(gpu, torch.bfloat16), y.to(gpu))
        lc.append(float(l1))
        lg.append(float(l2))
        if i == 0:
            cos = torch.nn.functional.cosine_similarity(o1.flatten().float(),
                                                        o2.cpu().flatten().float(), dim=0).item()
    gap = [abs(a - b) / abs(b) for a, b in zip(lg, lc)]
    print(f"lr {args.lr:g} b{batch:3d} {size:3d}px  logits cos {cos:.5f}  gpu {[round(v, 4) for v in lg]}  "
          f"cpu {[round(v, 4) for v in lc]}  max rel gap {max(gap) * 100:.2f} %", flush=True)
