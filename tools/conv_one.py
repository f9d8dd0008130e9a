#!/usr/bin/env python3
"""Run one conv pass (fwd / dgrad / wgrad) repeatedly under a chosen kernel mode — a target for
rocprofv3 counter collection.

  python tools/conv_one.py --mode 2 --op fwd --shape 256,14,512,512,3,2,1 --iters 20
  shape = N,H,Cin,Cout,k,stride,pad (square images)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=1)
    ap.add_argument("--op", default="fwd", choices=["fwd", "dgrad", "wgrad", "dgrad_bnstat",
                                                    "dgrad_reduce"])
    ap.add_argument("--shape", default="256,14,512,512,3,2,1")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--flip", action="store_true",
                    help="dgrad ops: pass the flipped filter (the dgrad-as-forward routes)")
    a = ap.parse_args()
    N, H, Cin, Cout, k, s, p = [int(v) for v in a.shape.split(",")]
    dev = torch.device("cuda")
    g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
    x = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
    w = torch.randn(Cout, k, k, Cin, device=dev, dtype=torch.bfloat16) * 0.05
    Ho, Wo = g.out_hw(H, H, k, k)
    dy = torch.randn(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
    ext().conv_set_glds_mode(a.mode)
    wf = None
    if a.flip and s == 1:
        wf = torch.empty(Cin, k, k, Cout, device=dev, dtype=torch.bfloat16)
        ext().conv_flip_weight(w, wf)
    if a.op in ("dgrad_bnstat", "dgrad_reduce"):
        # BN-backward statistics: fused into the dgrad epilogue vs dgrad + the BN reduce pass
        # (x plays the BN input; its ReLU bit mask and coefficients from a real BN forward)
        from tensorflowdistributedlearning_amd.ops import bn as B
        Cc = Cin
        coef = B.bn_finalize(B.bn_stats(x), x.numel() // Cc, torch.ones(Cc, device=dev),
                             torch.zeros(Cc, device=dev), torch.zeros(Cc, device=dev),
                             torch.ones(Cc, device=dev), 0.9, 1e-5, True)
        mask = torch.empty(x.numel() // 8, device=dev, dtype=torch.uint8)
        yb = B.bn_apply(x, coef, None, True, mask=mask)
        for _ in range(a.iters):
            if a.op == "dgrad_bnstat":
                C.conv_dgrad_bnstat(dy, w, x.shape, g, x, mask=mask, w_flip=wf)
            else:
                B.bn_bwd_reduce(C.conv_dgrad(dy, w, x.shape, g), yb, x, coef, 2)
        torch.cuda.synchronize()
        print("done", a.mode, a.op, a.shape)
        return
    for _ in range(a.iters):
        if a.op == "fwd":
            C.conv_fwd(x, w, g)
        elif a.op == "dgrad":
            C.conv_dgrad(dy, w, x.shape, g, w_flip=wf)
        else:
            C.conv_wgrad(dy, x, tuple(w.shape), g)
    torch.cuda.synchronize()
    print("done", a.mode, a.op, a.shape)


if __name__ == "__main__":
    main()
