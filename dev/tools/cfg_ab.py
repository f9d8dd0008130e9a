#!/usr/bin/env python3
"""A/B of the LDS-DMA conv tile configurations on given shapes (graph-timed, min over rounds):
0 = 256x128 / 8 waves / 3 stages, 1 = 256x64 / 4 waves, 2 = 128x128 / 4 waves / 4 stages,
3 = 128x128 / 2 stages (two workgroups per CU), 4 = 256x64 / 8 waves, 5 = 128x64 / 4 waves / 4
stages; "reg" = the register-staged kernel.  For the low-tile-count convs of the reference DeepLab
preset (13x13 feature maps at batch 64: 43 row tiles of 256).

  python dev/tools/cfg_ab.py [--op fwd|dgrad] [--shapes N,H,Cin,Cout,k,s,p[,d];...] [--cfgs 0,2,3,5,reg]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402
from route_ab import glds_cfg  # noqa: E402

SHAPES = ["64,13,512,512,3,1,2,2", "64,13,1024,256,1,1,0", "64,13,512,2048,1,1,0",
          "64,13,2048,512,1,1,0", "64,13,264,264,3,1,1", "64,13,256,256,3,1,4,4",
          "64,26,128,512,1,1,0", "64,26,512,128,1,1,0"]


def timed(fn):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(10):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 10 * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="fwd", choices=["fwd", "dgrad"])
    ap.add_argument("--shapes", default=";".join(SHAPES))
    ap.add_argument("--cfgs", default="0,2,3,5,reg")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for shp in a.shapes.split(";"):
        v = [int(t) for t in shp.split(",")]
        N, H, Cin, Cout, k, s, p = v[:7]
        d = v[7] if len(v) > 7 else 1
        g = C.ConvGeom((s, s), (p, p, p, p), (d, d))
        Ho, Wo = g.out_hw(H, H, k, k)
        x = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(Cout, k, k, Cin, device=dev, dtype=torch.bfloat16) * 0.05
        dy = torch.randn(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
        flop = 2.0 * N * Ho * Wo * Cout * Cin * k * k
        fn = (lambda: C.conv_fwd(x, w, g)) if a.op == "fwd" else (lambda: C.conv_dgrad(dy, w, x.shape, g))
        cfgs = a.cfgs.split(",")
        res = {c: [] for c in cfgs}
        for _ in range(a.rounds):
            for c in cfgs:
                glds_cfg(a.op, None)
                os.environ["TDL_GLDS_SLOTS"] = "512" if c == "3" else "256"
                if c == "reg":
                    ext().conv_set_glds_mode(0)
                else:
                    ext().conv_set_glds_mode(2)
                    glds_cfg(a.op, c)
                res[c].append(timed(fn))
        ext().conv_set_glds_mode(-1)
        glds_cfg(a.op, None)
        os.environ["TDL_GLDS_SLOTS"] = "256"
        best = min(res, key=lambda c: min(res[c]))
        print(f"{a.op} {shp:24s} " + " | ".join(f"cfg{c} {min(t):6.1f}us {flop / min(t) / 1e6:4.0f}TF"
                                                for c, t in res.items()) + f" | best {best}", flush=True)


if __name__ == "__main__":
    main()
