#!/usr/bin/env python3
"""Interleaved A/B timing of the LDS-DMA dgrad on ResNet-50 join shapes: plain overwrite, the
residual-join accumulate (dx += …), + the ReLU bit mask, and TDL_CONV_DBG ablations
(2 = skip MFMA, 128 = epilogue without global loads / stores).

  python dev/tools/dgrad_ablate.py [--rounds 5]

Needs a TDL_CONV_ABLATION=1 build of the extension (TDL_CONV_ABLATION=1 python build_ext.py
--force): production builds compile the TDL_CONV_DBG flags out."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402
from route_ab import glds_cfg  # noqa: E402

# (N, H, Cin, Cout, k, stride, pad): the conv whose dgrad writes dx [N, H, H, Cin]
SHAPES = ["256,56,256,64,1,1,0", "256,28,512,128,1,1,0", "256,14,1024,256,1,1,0",
          "256,7,2048,512,1,1,0", "256,56,64,64,3,1,1", "256,14,256,256,3,1,1",
          "256,56,128,128,3,2,1", "256,56,256,512,1,2,0"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shapes", default=";".join(SHAPES))
    ap.add_argument("--cfgs", action="store_true", help="also the 128x128 configurations")
    ap.add_argument("--dbg", default="", help="extra TDL_CONV_DBG values for plain dgrad, e.g. 1,64,129")
    a = ap.parse_args()
    dev = torch.device("cuda")
    ext().conv_set_glds_mode(-1)
    for shp in a.shapes.split(";"):
        N, H, Cin, Cout, k, s, p = [int(v) for v in shp.split(",")]
        g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
        Ho, Wo = g.out_hw(H, H, k, k)
        dy = torch.randn(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
        w = torch.randn(Cout, k, k, Cin, device=dev, dtype=torch.bfloat16) * 0.05
        prev = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        xin = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        mask = torch.randint(0, 256, (N * H * H * Cin // 8,), device=dev, dtype=torch.uint8)
        flop = 2.0 * N * Ho * Wo * Cout * Cin * k * k
        xs = (N, H, H, Cin)
        variants = [
            ("plain", 0, lambda: C.conv_dgrad(dy, w, xs, g)),
            ("acc", 0, lambda: C.conv_dgrad(dy, w, xs, g, out=prev, accumulate=True)),
            ("acc+mask", 0, lambda: C.conv_dgrad(dy, w, xs, g, out=prev, accumulate=True, mask=mask)),
            ("acc+mask noepimem", 128, lambda: C.conv_dgrad(dy, w, xs, g, out=prev, accumulate=True,
                                                          mask=mask)),
            ("plain nomfma", 2, lambda: C.conv_dgrad(dy, w, xs, g)),
            ("plain noepimem", 128, lambda: C.conv_dgrad(dy, w, xs, g)),
            ("fwd", 0, lambda: C.conv_fwd(xin, w, g)),
        ]
        for d in [int(v) for v in a.dbg.split(",") if v]:
            variants.append((f"plain dbg{d}", d, lambda: C.conv_dgrad(dy, w, xs, g)))
        if not a.cfgs:
            variants = [v for v in variants if v[0] != "plain nomfma"]
        variants += [] if not a.cfgs else [("plain cfg3x512", "cfg3", lambda: C.conv_dgrad(dy, w, xs, g)),
                     ("acc+mask cfg3x512", "cfg3", lambda: C.conv_dgrad(dy, w, xs, g, out=prev,
                                                                     accumulate=True, mask=mask)),
                     ("plain cfg2x512", "cfg2", lambda: C.conv_dgrad(dy, w, xs, g))]
        res = {v[0]: [] for v in variants}
        for _ in range(a.rounds):
            for name, dbg, fn in variants:
                cfg = dbg if isinstance(dbg, str) else None
                glds_cfg("dgrad", None)
                os.environ["TDL_GLDS_SLOTS"] = "256"
                if cfg:
                    glds_cfg("dgrad", cfg[3:])
                    os.environ["TDL_GLDS_SLOTS"] = "512"
                    dbg = 0
                os.environ["TDL_CONV_DBG"] = str(dbg)
                fn()
                torch.cuda.synchronize()
                # 10 calls captured as one graph: device time only (the Python/host path of a
                # call is ~100 us and would otherwise floor every fast variant)
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
                res[name].append(e0.elapsed_time(e1) / 10 * 1e3)
        os.environ["TDL_CONV_DBG"] = "0"
        mb = N * H * H * Cin * 2 / 1e6
        print(f"{shp:24s} dx {mb:6.1f}MB " + " | ".join(
            f"{n} {min(v):6.1f}us" for n, v in res.items()) + f" | {flop / min(res['plain']) / 1e6:.0f}TF plain",
            flush=True)


if __name__ == "__main__":
    main()
