#!/usr/bin/env python3
"""Per-shape conv microbenchmark: our MFMA implicit-GEMM kernels (fwd / dgrad / wgrad) on every
distinct ResNet-50 conv shape at a given batch, with MIOpen (torch channels_last bf16) timed on
the same box as a yardstick.  Interleaved rounds in one process (guide §5.4 rule 24).

  python bench/conv_bench.py --batch 256 --out gpurun_out/conv_bench.json
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402


def resnet50_shapes():
    """(name, H, W, Cin, Cout, k, stride, pad) with multiplicity."""
    out = {}

    def add(name, H, Cin, Cout, k, s, p):
        key = (H, Cin, Cout, k, s, p)
        if key in out:
            out[key][1] += 1
        else:
            out[key] = [name, 1]
    add("stem7x7", 224, 8, 64, 7, 2, 3)
    H, cin = 56, 64
    for i, n in enumerate((3, 4, 6, 3)):
        w = 64 * 2 ** i
        for j in range(n):
            s = 2 if (j == 0 and i > 0) else 1
            add(f"l{i+1}.conv1", H, cin, w, 1, 1, 0)
            add(f"l{i+1}.conv2", H, w, w, 3, s, 1)
            Ho = H // s
            add(f"l{i+1}.conv3", Ho, w, w * 4, 1, 1, 0)
            if j == 0:
                add(f"l{i+1}.down", H, cin, w * 4, 1, s, 0)
            H, cin = Ho, w * 4
    return [(v[0], v[1], *k) for k, v in out.items()]


def xception41_shapes():
    """Xception-41 at 299² (models/xception.py): every dense conv — the pointwise 1×1 convs of the
    separable blocks (26 of them at 19×19×728), the strided shortcuts and the stem."""
    return [("stem1", 1, 299, 8, 32, 3, 2, 1), ("stem2", 1, 150, 32, 64, 3, 1, 1),
            ("b1.pw1", 1, 150, 64, 128, 1, 1, 0), ("b1.pw2", 1, 150, 128, 128, 1, 1, 0),
            ("b1.pw3", 1, 75, 128, 128, 1, 1, 0), ("b1.sc", 1, 150, 64, 128, 1, 2, 0),
            ("b2.pw1", 1, 75, 128, 256, 1, 1, 0), ("b2.pw2", 1, 75, 256, 256, 1, 1, 0),
            ("b2.pw3", 1, 38, 256, 256, 1, 1, 0), ("b2.sc", 1, 75, 128, 256, 1, 2, 0),
            ("b3.pw1", 1, 38, 256, 728, 1, 1, 0), ("b3.pw2", 1, 38, 728, 728, 1, 1, 0),
            ("mid.pw", 26, 19, 728, 728, 1, 1, 0), ("b3.sc", 1, 38, 256, 728, 1, 2, 0),
            ("x1.pw2", 1, 19, 728, 1024, 1, 1, 0), ("x1.pw3", 1, 10, 1024, 1024, 1, 1, 0),
            ("x1.sc", 1, 19, 728, 1024, 1, 2, 0), ("x2.pw1", 1, 10, 1024, 1536, 1, 1, 0),
            ("x2.pw2", 1, 10, 1536, 1536, 1, 1, 0), ("x2.pw3", 1, 10, 1536, 2048, 1, 1, 0)]


def timeit(fn, iters=5):
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-miopen", action="store_true")
    ap.add_argument("--net", default="resnet50", choices=["resnet50", "xception41"])
    ap.add_argument("--gemm", action="store_true",
                    help="time the 1×1 convs' GEMMs with torch.mm (hipBLASLt) as a yardstick")
    ap.add_argument("--modes", default="1", help="comma list of conv kernel modes to time "
                    "(0 register-staged, 1 default selection, 2 LDS-DMA whenever aligned)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.batch
    rows = []
    tot = {"miopen": 0.0}
    modes = [int(m) for m in a.modes.split(",")]
    shapes = resnet50_shapes() if a.net == "resnet50" else xception41_shapes()
    tot["gemm"] = 0.0
    for name, mult, H, Cin, Cout, k, s, p in shapes:
        g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
        x = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(Cout, k, k, Cin, device=dev, dtype=torch.bfloat16) * 0.05
        Ho, Wo = g.out_hw(H, H, k, k)
        dy = torch.randn(N, Ho, Wo, Cout, device=dev, dtype=torch.bfloat16)
        flop = 2.0 * N * Ho * Wo * Cout * Cin * k * k
        st = torch.zeros(2, Cout, device=dev)
        r = dict(name=name, mult=mult, H=H, Cin=Cin, Cout=Cout, k=k, s=s, gflop=flop / 1e9)
        msg = f"{name:10s} x{mult} {H:3d}x{H:<3d} {Cin:4d}->{Cout:4d} k{k} s{s} |"
        for mode in modes:
            ext().conv_set_glds_mode(mode)
            t_f = timeit(lambda: C.conv_fwd(x, w, g, stats=st))
            t_d = timeit(lambda: C.conv_dgrad(dy, w, x.shape, g)) if name != "stem7x7" else 0.0
            t_w = timeit(lambda: C.conv_wgrad(dy, x, tuple(w.shape), g))
            r[f"m{mode}"] = dict(fwd_us=t_f, dgrad_us=t_d, wgrad_us=t_w)
            tot.setdefault(f"m{mode}", 0.0)
            tot[f"m{mode}"] += mult * (t_f + t_d + t_w)
            msg += (f" m{mode}: fwd {t_f:6.1f} ({flop / t_f / 1e6:4.0f}TF) dgrad {t_d:6.1f} "
                    f"wgrad {t_w:6.1f} ({flop / t_w / 1e6:4.0f}TF) |")
        ext().conv_set_glds_mode(-1)
        if a.gemm and k == 1 and s == 1:
            A = x.view(-1, Cin)
            W2 = w.view(Cout, Cin)
            D = dy.view(-1, Cout)
            g_f = timeit(lambda: torch.mm(A, W2.t()))
            g_d = timeit(lambda: torch.mm(D, W2))
            g_w = timeit(lambda: torch.mm(D.t(), A))
            r.update(gemm_fwd_us=g_f, gemm_dgrad_us=g_d, gemm_wgrad_us=g_w)
            tot["gemm"] += mult * (g_f + g_d + g_w)
            msg += f" mm fwd {g_f:6.1f} dgrad {g_d:6.1f} wgrad {g_w:6.1f}"
        if not a.no_miopen:
            xm = x.permute(0, 3, 1, 2)  # channels_last view
            wm = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            xm.requires_grad_(True)
            wm.requires_grad_(True)
            ym = F.conv2d(xm, wm, None, s, p)
            dym = dy.permute(0, 3, 1, 2)
            m_f = timeit(lambda: F.conv2d(xm, wm, None, s, p))
            m_b = timeit(lambda: torch.autograd.grad(ym, [xm, wm], dym, retain_graph=True))
            r.update(miopen_fwd_us=m_f, miopen_bwd_us=m_b)
            tot["miopen"] += mult * (m_f + m_b)
            msg += f" miopen fwd {m_f:6.1f} bwd {m_b:6.1f}"
        rows.append(r)
        print(msg, flush=True)
    print(json.dumps({k: round(v / 1e3, 2) for k, v in tot.items()}) + "  (ms per step, all convs; stem dgrad excluded for ours)")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"batch": N, "rows": rows, "total_ms": tot}, f, indent=1)


if __name__ == "__main__":
    main()
