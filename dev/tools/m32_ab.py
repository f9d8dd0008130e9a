#!/usr/bin/env python3
"""A/B of the 32×32×16-MFMA K loop (conv_glds_kernel M32) against the default 16×16×32 one on the
ResNet-50 convolutions that take the 256×128 FASTK LDS-DMA kernel at batch 1024: forward, and the
input gradient with transposed weights (conv_dgrad(w_t=...)).  Same process, interleaved rounds,
graph-timed (min over rounds); outputs are compared (bf16 rounding of different fp32 summation
orders only).

  python dev/tools/m32_ab.py [--batch 1024] [--rounds 3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402

# (name, H, Cin, Cout, k, stride, pad) at the conv's input resolution
SHAPES = [
    ("l2.conv3", 28, 128, 512, 1, 1, 0),
    ("l2.conv2", 28, 128, 128, 3, 1, 1),
    ("l3.conv1", 14, 1024, 256, 1, 1, 0),
    ("l3.conv2", 14, 256, 256, 3, 1, 1),
    ("l3.conv3", 14, 256, 1024, 1, 1, 0),
    ("l4.conv2", 7, 512, 512, 3, 1, 1),
    ("l4.conv3", 7, 512, 2048, 1, 1, 0),
    ("l4.conv1", 7, 2048, 512, 1, 1, 0),
    ("l3.conv2s2", 28, 256, 256, 3, 2, 1),
]


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    tot = {("fwd", 0): 0.0, ("fwd", 1): 0.0, ("dgrad", 0): 0.0, ("dgrad", 1): 0.0}
    for name, H, Ci, Co, k, s, p in SHAPES:
        N = args.batch
        g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
        x = torch.randn(N, H, H, Ci, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(Co, k, k, Ci, device=dev) / (k * k * Ci) ** 0.5).to(torch.bfloat16)
        wt = w.permute(1, 2, 3, 0).contiguous()
        Ho, Wo = g.out_hw(H, H, k, k)
        dy = torch.randn(N, Ho, Wo, Co, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * N * Ho * Wo * Co * Ci * k * k
        res = {}
        outs = {}
        for rnd in range(args.rounds):
            for m32 in (0, 1):
                ext().conv_set_m32(m32)
                tf = timed(lambda: C.conv_fwd(x, w, g))
                td = timed(lambda: C.conv_dgrad(dy, w, tuple(x.shape), g, w_t=wt))
                res[("fwd", m32)] = min(res.get(("fwd", m32), 1e9), tf)
                res[("dgrad", m32)] = min(res.get(("dgrad", m32), 1e9), td)
                if rnd == 0:
                    outs[m32] = (C.conv_fwd(x, w, g).float(),
                                 C.conv_dgrad(dy, w, tuple(x.shape), g, w_t=wt).float())
        ext().conv_set_m32(-1)
        ef = ((outs[0][0] - outs[1][0]).abs().max() / outs[0][0].abs().max()).item()
        ed = ((outs[0][1] - outs[1][1]).abs().max() / outs[0][1].abs().max()).item()
        line = f"{name:11s} {H:3d} {Ci:5d}->{Co:5d} k{k} s{s} |"
        for op in ("fwd", "dgrad"):
            a, b = res[(op, 0)], res[(op, 1)]
            tot[(op, 0)] += a
            tot[(op, 1)] += b
            line += (f" {op}: {a:7.1f} -> {b:7.1f} us ({(a / b - 1) * 100:+5.1f}%, "
                     f"{flops / b * 1e-6:5.0f} TF) |")
        line += f" rel diff fwd {ef:.1e} dgrad {ed:.1e}"
        print(line, flush=True)
        assert ef < 2e-2 and ed < 2e-2, (ef, ed)
    for op in ("fwd", "dgrad"):
        print(f"total {op}: {tot[(op, 0)]:.1f} -> {tot[(op, 1)]:.1f} us "
              f"({(tot[(op, 0)] / tot[(op, 1)] - 1) * 100:+.1f}%)")


if __name__ == "__main__":
    main()
