#!/usr/bin/env python3
"""Interleaved A/B timing of the weight-gradient kernels on ResNet-50 shapes: the default
selection, the LDS-DMA kernel forced on (conv_set_glds_mode(2)) with its configurations, and the
register-staged kernel (mode 0).  Reports µs per call and TFLOP/s.

  python dev/tools/wgrad_ab.py [--rounds 5] [--batch 256]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402
from route_ab import glds_cfg  # noqa: E402

# (H, Cin, Cout, k, stride, pad[, dilation]) of the conv whose weight gradient is taken (input H×H×Cin)
SHAPES = ["56,64,64,3,1,1", "28,128,128,3,1,1", "56,128,128,3,2,1", "14,256,256,3,1,1",
          "28,256,256,3,2,1", "7,512,512,3,1,1", "14,512,512,3,2,1", "56,64,64,1,1,0",
          "56,256,64,1,1,0", "56,64,256,1,1,0"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--shapes", default=";".join(SHAPES))
    ap.add_argument("--variants", default="default,gemm,glds0,glds2,glds3,glds0m8,glds0m32")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.batch
    variants = {
        "default": (1, {}), "gemm": (0, {}),
        "glds0": (2, {"cfg": "0"}), "glds2": (2, {"cfg": "2"}),
        "glds3": (2, {"cfg": "3", "TDL_GLDS_SLOTS": "512"}),
        "glds1": (2, {"cfg": "1"}), "glds5": (2, {"cfg": "5"}),
        "glds0m8": (2, {"cfg": "0", "TDL_GLDS_WGRAD_MINSTEPS": "8"}),
        "glds0m32": (2, {"cfg": "0", "TDL_GLDS_WGRAD_MINSTEPS": "32"}),
        "glds2m8": (2, {"cfg": "2", "TDL_GLDS_WGRAD_MINSTEPS": "8"}),
    }
    names = a.variants.split(",")
    keys = sorted({k for _, e in variants.values() for k in e if k != "cfg"})
    for shp in a.shapes.split(";"):
        v = [int(t) for t in shp.split(",")]
        H, Cin, Cout, k, s, p = v[:6]
        d = v[6] if len(v) > 6 else 1
        g = C.ConvGeom((s, s), (p, p, p, p), (d, d))
        Ho, Wo = g.out_hw(H, H, k, k)
        x = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
        out = torch.empty(Cout, k, k, Cin, device=dev, dtype=torch.float32)
        flop = 2.0 * N * Ho * Wo * Cout * Cin * k * k
        res = {n: [] for n in names}
        ref = None
        for _ in range(a.rounds):
            for n in names:
                mode, env = variants[n]
                for kk in keys:
                    os.environ.pop(kk, None)
                os.environ.update({kk: vv for kk, vv in env.items() if kk != "cfg"})
                glds_cfg("wgrad", env.get("cfg"))
                ext().conv_set_glds_mode(mode)
                C.conv_wgrad(dy, x, out.shape, g, out=out)
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                else:
                    err = ((out - ref).norm() / ref.norm()).item()
                    assert err < 1e-3, (shp, n, err)
                e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                e0.record()
                for _ in range(10):
                    C.conv_wgrad(dy, x, out.shape, g, out=out)
                e1.record()
                torch.cuda.synchronize()
                res[n].append(e0.elapsed_time(e1) / 10 * 1e3)
        for kk in keys:
            os.environ.pop(kk, None)
        glds_cfg("wgrad", None)
        ext().conv_set_glds_mode(-1)
        best = min(res, key=lambda n: min(res[n]))
        print(f"{shp:18s} " + " | ".join(f"{n} {min(v):6.1f}us {flop / min(v) / 1e6:4.0f}TF"
                                         for n, v in res.items()) + f" | best {best}", flush=True)


if __name__ == "__main__":
    main()
