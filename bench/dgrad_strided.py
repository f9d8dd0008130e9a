#!/usr/bin/env python3
"""Stride-2 input gradients of ResNet-50 (b1024 by default): the DGRAD kernel (parity classes)
vs the same dx computed as one stride-1 FORWARD conv of dy per parity class (a, b) with that
class's flipped sub-filter — class (a, b) of dx (pixels h = a + 2i, w = b + 2j) only receives the
taps r ≡ a + ph (mod 2), s ≡ b + pw (mod 2), so it is a Th×Tw forward conv over dy with padding
Th − 1 − (a + ph − r0)/2.  Times each, checks the assembled dx against the DGRAD kernel.

python bench/dgrad_strided.py [--batch 1024]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402

SHAPES = [  # (name, H_in, Cin, Cout, k, pad)
    ("l2.conv2 3x3 s2 128", 56, 128, 128, 3, 1),
    ("l3.conv2 3x3 s2 256", 28, 256, 256, 3, 1),
    ("l4.conv2 3x3 s2 512", 14, 512, 512, 3, 1),
    ("l2.down 1x1 s2 256->512", 56, 256, 512, 1, 0),
    ("l3.down 1x1 s2 512->1024", 28, 512, 1024, 1, 0),
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


def classes(k, pad, H, s=2):
    """per class (a, b): (r0, Th, pad', Hc) for rows (columns alike)"""
    out = []
    for a in range(s):
        r0 = (a + pad) % s
        Th = (k - r0 + s - 1) // s if r0 < k else 0
        e = (a + pad - r0) // s
        Hc = (H - a + s - 1) // s
        out.append((a, r0, Th, Th - 1 - e, Hc))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.batch
    for name, H, Cin, Cout, k, p in SHAPES:
        g = C.ConvGeom((2, 2), (p, p, p, p), (1, 1))
        Ho, Wo = g.out_hw(H, H, k, k)
        torch.manual_seed(0)
        w = (torch.randn(Cout, k, k, Cin, device=dev) * 0.05).bfloat16()
        dy = torch.randn(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
        xs = (N, H, H, Cin)
        t_d = timed(lambda: C.conv_dgrad(dy, w, xs, g))
        ref = C.conv_dgrad(dy, w, xs, g)
        cl = classes(k, p, H)
        jobs = []
        for (ra, r0, Th, pr, Hc) in cl:
            for (cb, s0, Tw, pc, Wc) in cl:
                if Th == 0 or Tw == 0:
                    continue
                rr = [r0 + 2 * (Th - 1 - t) for t in range(Th)]
                ss = [s0 + 2 * (Tw - 1 - u) for u in range(Tw)]
                wsub = w[:, rr][:, :, ss].permute(3, 1, 2, 0).contiguous()  # [Cin, Th, Tw, Cout]
                gg = C.ConvGeom((1, 1), (pr, Th - 1 - pr + (Hc - Ho), pc, Tw - 1 - pc + (Wc - Wo)), (1, 1))
                y = torch.empty(N, Hc, Wc, Cin, device=dev, dtype=torch.bfloat16)
                jobs.append((ra, cb, wsub, pr, pc, Hc, Wc, y))

        def run():
            for (ra, cb, wsub, pr, pc, Hc, Wc, y) in jobs:
                ext().conv_fwd(dy, wsub, y, None, None, 1, 1, pr, pc, 1, 1, False)
        t_c = timed(run)
        run()
        dx = torch.zeros(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        for (ra, cb, wsub, pr, pc, Hc, Wc, y) in jobs:
            dx[:, ra::2, cb::2] = y
        err = ((dx.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        print(f"{name:26s} dgrad {t_d:7.1f} us   per-class forwards {t_c:7.1f} us ({len(jobs)} launches)"
              f"   rel err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
