"""BN backward reduction at ResNet-50 b256 shapes: µs and TB/s per shape (A/B of the reduce
variants via TDL_BN_RED_* env knobs, which are read once per process).
  TDL_BN_RED_PART=1 TDL_BN_RED_NT=512 python dev/tools/bn_red_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import bn as B  # noqa: E402


def t(fn, it=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


dev = "cuda"
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("TDL_BN_RED"))
tot = 0.0
for (hw, C, n) in [(112, 64, 1), (56, 64, 6), (56, 256, 3), (56, 128, 1), (28, 128, 7),
                   (28, 512, 4), (14, 256, 11), (14, 1024, 6), (7, 512, 5), (7, 2048, 3)]:
    M = 256 * hw * hw
    x = torch.randn(M, C, device=dev).bfloat16()
    dy = torch.randn(M, C, device=dev).bfloat16()
    coef = torch.stack([torch.rand(C) + .5, torch.randn(C), torch.randn(C) * .1,
                        torch.rand(C) + .5]).to(dev)
    ref = B.bn_bwd_reduce(dy, None, x, coef, 2)
    tr = t(lambda: B.bn_bwd_reduce(dy, None, x, coef, 2))
    mb = M * C * 2 / 1e6
    tot += n * tr
    print(f"{tag:40s} M={M:8d} C={C:5d} reduce {tr:7.1f}us ({2 * mb / tr:5.2f} TB/s) x{n}",
          flush=True)
    del x, dy
print(f"{tag:40s} weighted total {tot / 1e3:.3f} ms", flush=True)
