#!/usr/bin/env python3
"""Probe strided-dgrad timing: the parity-class dgrad vs the equivalent dense sub-GEMM."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402


def t(fn, it=10):
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


dev = torch.device("cuda")
N = 256
for (H, Cin, Cout, k, s, p) in [(56, 256, 512, 1, 2, 0), (28, 512, 1024, 1, 2, 0),
                                (14, 512, 512, 3, 2, 1), (56, 128, 128, 3, 2, 1)]:
    g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
    Ho = (H + 2 * p - k) // s + 1
    w = torch.randn(Cout, k, k, Cin, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(N, Ho, Ho, Cout, device=dev, dtype=torch.bfloat16)
    res = {}
    for tpb in ("1", "2", "4"):
        os.environ["TDL_CONV_TPB"] = tpb
        res[f"tpb{tpb}"] = t(lambda: C.conv_dgrad(dy, w, (N, H, H, Cin), g))
    os.environ.pop("TDL_CONV_TPB")
    # dense equivalent: stride-1 dgrad onto the Ho x Ho grid (the class-0 GEMM)
    g1 = C.ConvGeom((1, 1), (p, p, p, p), (1, 1))
    dense = t(lambda: C.conv_dgrad(dy, w, (N, Ho, Ho, Cin), g1))
    zero = t(lambda: torch.zeros(N, H, H, Cin, device=dev, dtype=torch.bfloat16))
    print(f"H{H} {Cin}->{Cout} k{k} s{s}: " + " ".join(f"{k_}={v:.1f}us" for k_, v in res.items())
          + f" | dense(stride1 on Ho grid)={dense:.1f}us  zeros(dx)={zero:.1f}us", flush=True)
