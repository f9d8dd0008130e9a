#!/usr/bin/env python3
"""Where does a K-step of the LDS-DMA conv kernel go?  Graph-timed forward (or dgrad) of one
shape under TDL_CONV_DBG ablations: 1 = operand loads out of range (the DMA still runs, no
memory traffic), 2 = no MFMA, 16 = no LDS fragment reads, 32 = no barrier, 64 = no DMA at all,
128 = epilogue without global memory.  Timing-only: the results are wrong.

  python dev/tools/fwd_ablate.py [--op fwd|dgrad] [--shapes N,H,Cin,Cout,k,s,p;...] [--dbg 0,1,2,...]

Needs a TDL_CONV_ABLATION=1 build of the extension (TDL_CONV_ABLATION=1 python build_ext.py
--force): production builds compile the TDL_CONV_DBG flags out."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402

SHAPES = ["256,14,256,256,3,1,1", "256,28,128,128,3,1,1", "256,56,64,256,1,1,0"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="fwd", choices=["fwd", "dgrad"])
    ap.add_argument("--shapes", default=";".join(SHAPES))
    ap.add_argument("--dbg", default="0,1,2,16,32,64,18,66,80,194,210")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for shp in a.shapes.split(";"):
        N, H, Cin, Cout, k, s, p = [int(v) for v in shp.split(",")]
        g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
        Ho, Wo = g.out_hw(H, H, k, k)
        x = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(Cout, k, k, Cin, device=dev, dtype=torch.bfloat16) * 0.05
        dy = torch.randn(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
        flop = 2.0 * N * Ho * Wo * Cout * Cin * k * k
        fn = (lambda: C.conv_fwd(x, w, g)) if a.op == "fwd" else (lambda: C.conv_dgrad(dy, w, x.shape, g))
        dbgs = [int(v) for v in a.dbg.split(",")]
        res = {d: [] for d in dbgs}
        for _ in range(a.rounds):
            for d in dbgs:
                os.environ["TDL_CONV_DBG"] = str(d)
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
                res[d].append(e0.elapsed_time(e1) / 10 * 1e3)
        os.environ["TDL_CONV_DBG"] = "0"
        print(f"{a.op} {shp:22s} " + " | ".join(f"dbg{d} {min(v):6.1f}us" for d, v in res.items())
              + f" | {flop / min(res[dbgs[0]]) / 1e6:.0f} TF/s at dbg{dbgs[0]}", flush=True)


if __name__ == "__main__":
    main()
