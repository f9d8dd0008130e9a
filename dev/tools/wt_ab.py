#!/usr/bin/env python3
"""Dgrad with the weights as [K,R,S,C] (transposed LDS reads of the B operand) vs a [R,S,C,K]
copy (K-contiguous rows, ds_read_b128): graph-timed A/B in one process, bitwise result check.

  python dev/tools/wt_ab.py [--shapes N,H,Cin,Cout,k,s,p;...]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402

SHAPES = ["256,14,256,256,3,1,1", "256,28,128,128,3,1,1", "256,56,256,64,1,1,0",
          "256,28,512,128,1,1,0", "256,14,1024,256,1,1,0", "256,7,2048,512,1,1,0",
          "256,56,128,128,3,2,1", "256,56,64,256,1,1,0"]


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
    ap.add_argument("--shapes", default=";".join(SHAPES))
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for shp in a.shapes.split(";"):
        N, H, Cin, Cout, k, s, p = [int(v) for v in shp.split(",")]
        g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
        Ho, Wo = g.out_hw(H, H, k, k)
        w = torch.randn(Cout, k, k, Cin, device=dev, dtype=torch.bfloat16) * 0.05
        wt = w.permute(1, 2, 3, 0).contiguous()
        dy = torch.randn(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
        xs = (N, H, H, Cin)
        r0 = C.conv_dgrad(dy, w, xs, g)
        r1 = C.conv_dgrad(dy, w, xs, g, w_t=wt)
        same = torch.equal(r0, r1)
        res = {"w": [], "w_t": []}
        for _ in range(a.rounds):
            res["w"].append(timed(lambda: C.conv_dgrad(dy, w, xs, g)))
            res["w_t"].append(timed(lambda: C.conv_dgrad(dy, w, xs, g, w_t=wt)))
        print(f"{shp:24s} w {min(res['w']):7.1f}us | w_t {min(res['w_t']):7.1f}us | bitwise equal {same}",
              flush=True)


if __name__ == "__main__":
    main()
