#!/usr/bin/env python3
"""Time every input-gradient (or, --op fwd, forward) route row (csrc/kernels/conv_route.hip) that
takes a given conv, forced one at a time (conv_route_force), plain and with the fused BN sums,
and check each against the default row's result.

  python dev/tools/dgrad_rows.py --shape N,H,Cin,Cout,k,s,p [--stats] [--op fwd]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="128,150,32,64,3,1,1")
    ap.add_argument("--stats", action="store_true")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--op", default="dgrad", choices=["dgrad", "fwd", "wgrad"])
    ap.add_argument("--rows", default="", help="only these rows (comma list), timed interleaved")
    ap.add_argument("--rounds", type=int, default=1)
    a = ap.parse_args()
    e = ext()
    dev = torch.device("cuda")
    N, H, Cin, Cout, k, s, p = [int(t) for t in a.shape.split(",")]
    g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
    Ho, _ = g.out_hw(H, H, k, k)
    torch.manual_seed(0)
    w = (torch.randn(Cout, k, k, Cin, device=dev) / (k * Cout) ** 0.5).bfloat16()
    dy = torch.randn(N, Ho, Ho, Cout, device=dev).bfloat16()
    x = torch.randn(N, H, H, Cin, device=dev).bfloat16()
    if s > 1:
        wf = C.flip_classes(w, g)
    else:
        wf = torch.empty(Cin, k, k, Cout, device=dev, dtype=torch.bfloat16)
        e.conv_flip_weight(w, wf)
    fwd = a.op == "fwd"
    dx = torch.empty_like(dy) if fwd else torch.empty_like(x)
    if a.op == "wgrad":
        dx = torch.empty(Cout, k, k, Cin, device=dev, dtype=torch.float32)
    red = torch.zeros(2, Cout if fwd else Cin, device=dev)
    args = (g.stride[0], g.stride[1], g.padding[0], g.padding[2], 1, 1)
    opi = {"fwd": 0, "dgrad": 1, "wgrad": 2}[a.op]

    def run():
        red.zero_()
        if a.op == "wgrad":
            return e.conv_wgrad(dy, x, dx, None, *args, False, None)
        if fwd:
            return e.conv_fwd(x, w, dx, None, red if a.stats else None, *args, False)
        return e.conv_dgrad(dy, w, dx, *args, False, None, None, x if a.stats else None,
                            red if a.stats else None, None, wf)

    run()
    torch.cuda.synchronize()
    ref = dx.float().clone()
    default = e.conv_last_route(opi)
    flop = 2.0 * N * Ho * Ho * Cout * Cin * k * k
    names = [r["name"] for r in e.conv_route_table() if r["op"] == a.op]
    if a.rows:
        names = [n for n in a.rows.split(",") if n in names]
    best, errs, fails = {}, {}, {}
    for _ in range(a.rounds):  # (rounds interleave the rows: no clock-ramp bias for late rows)
        for name in names:
            if name in fails:
                continue
            e.conv_route_force(opi, name)
            try:
                run()
                torch.cuda.synchronize()
                errs[name] = ((dx.float() - ref).norm() / ref.norm()).item()
                e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.iters
                best[name] = min(best.get(name, us), us)
            except RuntimeError as ex:
                fails[name] = str(ex).split("\n")[0][:60]
            finally:
                e.conv_route_force(opi, "")
    for name in names:
        if name in fails:
            print(f"{name:30s}   -  ({fails[name]})", flush=True)
        elif name in best:
            us = best[name]
            tag = " (default)" if name == default else ""
            print(f"{name:30s} {us:8.1f} us {flop / us / 1e6:6.0f} TF/s  err {errs[name]:.1e}{tag}",
                  flush=True)


if __name__ == "__main__":
    main()
