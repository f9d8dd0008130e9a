#!/usr/bin/env python3
"""Stride-1 dgrad paths per ResNet-50 shape (b1024 by default), standalone kernels:

  dgrad       default conv_dgrad (LDS-DMA DGRAD mode, weights through the transposed-read path)
  dgrad_wt    conv_dgrad with the [R,S,C,K] weight copy (K-contiguous B rows)
  as_fwd      the same product as a FORWARD conv of dy with the flipped filter
              w'[c, r', s', k] = w[k, R−1−r', S−1−s', c] and padding (R−1)·d − p — i.e. what a
              dgrad routed through the forward kernels (LDS-DMA / producer-consumer) would cost
  fwd         the layer's own forward, for scale

python bench/dgrad_paths.py [--batch 1024]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402

SHAPES = [  # (name, H, Cin, Cout, k)
    ("l1.conv2 3x3 64", 56, 64, 64, 3),
    ("l2.conv2 3x3 128", 28, 128, 128, 3),
    ("l3.conv2 3x3 256", 14, 256, 256, 3),
    ("l4.conv2 3x3 512", 7, 512, 512, 3),
    ("l1.conv3 1x1 64->256", 56, 64, 256, 1),
    ("l3.conv1 1x1 1024->256", 14, 1024, 256, 1),
    ("l3.conv3 1x1 256->1024", 14, 256, 1024, 1),
    ("l4.conv3 1x1 512->2048", 7, 512, 2048, 1),
]


def timed(fn, iters=5, rounds=3):
    out = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / iters)
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.batch
    for name, H, Cin, Cout, k in SHAPES:
        p = (k - 1) // 2
        g = C.ConvGeom((1, 1), (p, p, p, p), (1, 1))
        gf = C.ConvGeom((1, 1), (k - 1 - p, k - 1 - p, k - 1 - p, k - 1 - p), (1, 1))
        torch.manual_seed(0)
        x = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(Cout, k, k, Cin, device=dev) * 0.05).bfloat16()
        dy = torch.randn(N, H, H, Cout, device=dev, dtype=torch.bfloat16)
        w_t = w.permute(1, 2, 3, 0).contiguous()                       # [R, S, C, K]
        w_f = w.flip(1, 2).permute(3, 1, 2, 0).contiguous()            # [C, R, S, K] flipped
        dx = torch.empty_like(x)
        y = torch.empty(N, H, H, Cout, device=dev, dtype=torch.bfloat16)
        args = (1, 1, p, p, 1, 1)
        fargs = (1, 1, k - 1 - p, k - 1 - p, 1, 1)
        t_d = timed(lambda: ext().conv_dgrad(dy, w, dx, *args, False, None, None))
        t_dt = timed(lambda: ext().conv_dgrad(dy, w, dx, *args, False, None, w_t))
        t_af = timed(lambda: ext().conv_fwd(dy, w_f, dx, None, None, *fargs, False))
        t_f = timed(lambda: ext().conv_fwd(x, w, y, None, None, *args, False))
        ref = C.conv_dgrad(dy, w, x.shape, g)
        alt = torch.empty_like(x)
        ext().conv_fwd(dy, w_f, alt, None, None, *fargs, False)
        err = ((alt.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        print(f"{name:26s} dgrad {t_d:7.1f}  dgrad_wt {t_dt:7.1f}  as_fwd {t_af:7.1f}  fwd {t_f:7.1f} us"
              f"   (as_fwd vs dgrad rel {err:.1e})", flush=True)


if __name__ == "__main__":
    main()
