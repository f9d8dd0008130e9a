#!/usr/bin/env python3
"""Folded BN + ReLU (ops/bnconv.py) vs the materialised BN per ResNet-50 bottleneck shape, b1024,
standalone kernels (median of interleaved rounds):

  fwd    bn_apply(z) → u (+ bit mask) + conv_fwd(u)      vs  conv_fwd(z, aff)
  dgrad  bit-mask dgrad with fused BN sums                vs  aff-mask dgrad with fused BN sums
  wgrad  conv_wgrad(dy, u)                                vs  conv_wgrad(dy, z, aff)

python bench/bnconv_ab.py [--batch 1024] [--iters 5] [--rounds 3]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflowdistributedlearning_amd.ops import conv as C, bn as B  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402

# (name, H, Cin, Cout, k, stride, count per step)
SHAPES = [
    ("l1.conv2 3x3 64", 56, 64, 64, 3, 1, 3),
    ("l1.conv3 1x1 64->256", 56, 64, 256, 1, 1, 3),
    ("l2.conv2 3x3 128 s2", 56, 128, 128, 3, 2, 1),
    ("l2.conv2 3x3 128", 28, 128, 128, 3, 1, 3),
    ("l2.conv3 1x1 128->512", 28, 128, 512, 1, 1, 4),
    ("l3.conv2 3x3 256 s2", 28, 256, 256, 3, 2, 1),
    ("l3.conv2 3x3 256", 14, 256, 256, 3, 1, 5),
    ("l3.conv3 1x1 256->1024", 14, 256, 1024, 1, 1, 6),
    ("l4.conv2 3x3 512 s2", 14, 512, 512, 3, 2, 1),
    ("l4.conv2 3x3 512", 7, 512, 512, 3, 1, 2),
    ("l4.conv3 1x1 512->2048", 7, 512, 2048, 1, 1, 3),
]


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.batch
    tot = {"fwd": [0, 0], "dgrad": [0, 0], "wgrad": [0, 0]}
    for name, H, Cin, Cout, k, s, cnt in SHAPES:
        if a.only and a.only not in name:
            continue
        p = (k - 1) // 2
        g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
        args = (s, s, p, p, 1, 1)
        torch.manual_seed(0)
        z = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(Cout, k, k, Cin, device=dev) * 0.05).bfloat16()
        coef = torch.zeros(4, Cin, device=dev)
        coef[0].uniform_(0.5, 1.5)
        coef[1].normal_(0, 0.5)
        Ho, Wo = g.out_hw(H, H, k, k)
        y = torch.empty(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
        st = torch.zeros(2, Cout, device=dev)
        mask = torch.empty(z.numel() // 8, device=dev, dtype=torch.uint8)
        u = B.bn_apply(z, coef, None, True, mask=mask)
        dx = torch.empty_like(z)
        red = torch.zeros(2, Cin, device=dev)
        dw = torch.empty(Cout, k, k, Cin, device=dev)

        def f0():
            B.bn_apply(z, coef, None, True, mask=mask)
            ext().conv_fwd(u, w, y, None, st, *args, False)

        def f1():
            ext().conv_fwd(z, w, y, None, st, *args, False, None, coef)

        def d0():
            ext().conv_dgrad(dy, w, dx, *args, False, mask, None, z, red)

        def d1():
            ext().conv_dgrad(dy, w, dx, *args, False, None, None, z, red, coef)

        def w0():
            ext().conv_wgrad(dy, u, dw, None, *args, False)

        def w1():
            ext().conv_wgrad(dy, z, dw, None, *args, False, coef)

        res = {kk: [] for kk in ("f0", "f1", "d0", "d1", "w0", "w1")}
        for _ in range(a.rounds):
            for kk, fn in (("f0", f0), ("f1", f1), ("d0", d0), ("d1", d1), ("w0", w0), ("w1", w1)):
                res[kk].append(timed(fn, a.iters))
        m = {kk: statistics.median(v) for kk, v in res.items()}
        print(f"{name:26s} x{cnt}  fwd {m['f0']:7.1f} -> {m['f1']:7.1f} us   dgrad {m['d0']:7.1f} -> "
              f"{m['d1']:7.1f}   wgrad {m['w0']:7.1f} -> {m['w1']:7.1f}", flush=True)
        for key, (x0, x1) in (("fwd", ("f0", "f1")), ("dgrad", ("d0", "d1")), ("wgrad", ("w0", "w1"))):
            tot[key][0] += cnt * m[x0]
            tot[key][1] += cnt * m[x1]
    for key, (t0, t1) in tot.items():
        print(f"per step {key:5s} {t0 / 1e3:6.2f} -> {t1 / 1e3:6.2f} ms")
    print(f"per step total {sum(v[0] for v in tot.values()) / 1e3:6.2f} -> "
          f"{sum(v[1] for v in tot.values()) / 1e3:6.2f} ms")


if __name__ == "__main__":
    main()
