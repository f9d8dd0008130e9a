"""Depthwise 3×3 forward / dgrad / wgrad at Xception-41 b128 shapes: µs and HBM-equivalent TB/s
(wgrad: the tile kernel vs the sliding-window kernel, TDL_DW_WG_TILE=0, same process)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd.ops import conv as C  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


for (hw, c) in [(19, 728), (150, 128), (75, 256), (38, 728)]:
    x = torch.randn(128, hw, hw, c, device="cuda").bfloat16()
    w = (torch.randn(3, 3, c, device="cuda") * 0.3).bfloat16()
    y = torch.empty_like(x)
    f = lambda: ext().dwconv_fwd(x, w, None, y, 1, 1, 1, 1, 1, 1, False, False)
    d = lambda: ext().dwconv_dgrad(x, w, y, 1, 1, 1, 1, 1, 1, None)
    mb = x.numel() * 2 / 1e6
    tf, td = t(f), t(d)
    gw = torch.zeros(3, 3, c, device="cuda")
    wg = lambda: ext().dwconv_wgrad(y, x, gw, None, 1, 1, 1, 1, 1, 1, False, False)
    res = {}
    for on in ("0", "1", "0", "1"):
        os.environ["TDL_DW_WG_TILE"] = on
        res.setdefault(on, []).append(t(wg))
    os.environ.pop("TDL_DW_WG_TILE", None)
    w0, w1 = min(res["0"]), min(res["1"])
    print(f"{hw}x{hw}x{c}: fwd {tf:7.1f} us ({2 * mb / tf:4.2f} TB/s)  dgrad {td:7.1f} us "
          f"({2 * mb / td:4.2f} TB/s)  wgrad slide {w0:7.1f} -> tile {w1:7.1f} us "
          f"({2 * mb / w1:4.2f} TB/s)", flush=True)
    del x, y

# stride-2 input gradients (Xception's strided separable convs, fixed padding 1): the 2x2-block
# kernel vs the row kernel (TDL_DW_S2_OFF=1), same process
for (hw, c) in [(150, 128), (75, 256), (38, 728), (19, 1024)]:
    ho = (hw + 2 - 3) // 2 + 1
    dy = torch.randn(128, ho, ho, c, device="cuda").bfloat16()
    w = (torch.randn(3, 3, c, device="cuda") * 0.3).bfloat16()
    dx = torch.empty(128, hw, hw, c, device="cuda").bfloat16()
    d = lambda: ext().dwconv_dgrad(dy, w, dx, 2, 2, 1, 1, 1, 1, None)
    res = {}
    for off in (1, 0, 1, 0):
        if off:
            os.environ["TDL_DW_S2_OFF"] = "1"
        else:
            os.environ.pop("TDL_DW_S2_OFF", None)
        res.setdefault(off, []).append(t(d))
    mb = (dx.numel() + dy.numel()) * 2 / 1e6
    a, b = min(res[1]), min(res[0])
    print(f"s2 dgrad {hw}x{hw}x{c}: rows {a:7.1f} us ({mb / a:4.2f} TB/s) -> 2x2 blocks {b:7.1f} us "
          f"({mb / b:4.2f} TB/s)", flush=True)
    del dy, dx

# stride-2 forward / weight gradient: the tile kernels vs the row kernels (TDL_DW_S2_TILE=0)
for (hw, c) in [(150, 128), (75, 256), (38, 728), (19, 1024)]:
    ho = (hw + 2 - 3) // 2 + 1
    x = torch.randn(128, hw, hw, c, device="cuda").bfloat16()
    w = (torch.randn(3, 3, c, device="cuda") * 0.3).bfloat16()
    y = torch.empty(128, ho, ho, c, device="cuda").bfloat16()
    gw = torch.zeros(3, 3, c, device="cuda")
    f = lambda: ext().dwconv_fwd(x, w, None, y, 2, 2, 1, 1, 1, 1, False, False)
    g = lambda: ext().dwconv_wgrad(y, x, gw, None, 2, 2, 1, 1, 1, 1, False, False)
    res = {}
    for on in ("0", "1", "0", "1"):
        os.environ["TDL_DW_S2_TILE"] = on
        res.setdefault(on, []).append((t(f), t(g)))
    os.environ.pop("TDL_DW_S2_TILE", None)
    (f0, g0), (f1, g1) = (min(v) for v in (res["0"], res["1"]))
    mb = (x.numel() + y.numel()) * 2 / 1e6
    print(f"s2 {hw}x{hw}x{c}: fwd rows {f0:7.1f} -> tile {f1:7.1f} us ({mb / f1:4.2f} TB/s)  "
          f"wgrad rows {g0:7.1f} -> tile {g1:7.1f} us", flush=True)
    del x, y
