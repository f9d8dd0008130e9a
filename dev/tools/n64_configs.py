"""A/B of conv kernel configurations for the 64-output-channel ResNet-50 layer1 convs (fwd and
dgrad): register-staged (reg) vs LDS-DMA configs (route_ab.glds_cfg: 1 = 256x64/4 waves,
4 = 256x64/8 waves, 5 = 128x64/4 waves/4 stages).  Interleaved rounds, min over rounds.
  python dev/tools/n64_configs.py [--batch 256]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402
from route_ab import glds_cfg  # noqa: E402

SHAPES = [(56, 64, 64, 3, 1, 1), (56, 64, 64, 1, 1, 0), (56, 256, 64, 1, 1, 0),
          (28, 128, 128, 3, 1, 1)]


def t(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for H, cin, cout, k, s, p in SHAPES:
        g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
        x = torch.randn(a.batch, H, H, cin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(cout, k, k, cin, device=dev, dtype=torch.bfloat16) * 0.05
        Ho, Wo = g.out_hw(H, H, k, k)
        dy = torch.randn(a.batch, Ho, Wo, cout, device=dev, dtype=torch.bfloat16)
        res = {}
        for _ in range(a.rounds):
            for name, mode, cfg in (("reg", 0, None), ("g1", 2, 1), ("g4", 2, 4), ("g5", 2, 5)):
                ext().conv_set_glds_mode(mode)
                for op in ("fwd", "dgrad"):
                    glds_cfg(op, cfg)
                    fn = (lambda: C.conv_fwd(x, w, g)) if op == "fwd" else \
                        (lambda: C.conv_dgrad(dy, w, x.shape, g))
                    res.setdefault((name, op), []).append(t(fn))
        ext().conv_set_glds_mode(-1)
        print(f"{H}x{H} {cin}->{cout} k{k}: " + "  ".join(
            f"{n}/{o} {min(v):6.1f}" for (n, o), v in res.items()), flush=True)


if __name__ == "__main__":
    main()
