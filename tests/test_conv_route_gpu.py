"""Every row of the conv route table (csrc/kernels/conv_route.hip) — defaults, opt-in rows and the
rows the kernel tests use — forced onto a problem inside its shape window and checked against the
fp32 oracle.  A forced row whose kernel does not take the problem, or whose
tile config the launcher does not instantiate, raises in the launcher and fails here; the launcher
must also report that it ran exactly that row (``conv_last_route``).

The reference has one cuDNN conv call per layer and no routing (model.py:56-63 →
tf.layers.conv2d); the table is this framework's own dispatch, so parity here is vs the fp32
oracle of the same op."""
import math
import zlib

import pytest
import torch

from tensorflowdistributedlearning_amd.ops import conv as C
from tensorflowdistributedlearning_amd.ops import bn as B

pytestmark = pytest.mark.gpu

RF_STATS, RF_JOIN, RF_AFF, RF_FP8, RF_WFLIP, RF_STRIDED = 1, 2, 4, 8, 64, 256
OPS = {"fwd": 0, "dgrad": 1, "wgrad": 2}


def _table():
    try:
        from tensorflowdistributedlearning_amd import _native
        return _native.load().conv_route_table()
    except Exception:  # (collection without the extension: the gpu marker skips anyway)
        return []


ROWS = _table()


def _ext():
    from tensorflowdistributedlearning_amd.ops.common import ext
    return ext()


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


def _pick(lo, hi):
    """a channel count inside [lo, hi]: 64-aligned where the window allows (the LDS-DMA / halo /
    producer-consumer kernels' FASTK alignment), else the largest multiple of 8 in it."""
    v = -(-max(lo, 64) // 64) * 64
    return v if v <= hi else (hi // 8) * 8


def _problem(r):
    t0, t1 = r["taps"]
    k = 3 if t0 <= 9 <= t1 else 1 if t0 <= 1 else int(math.isqrt(t0))
    return k, _pick(*r["cin"]), _pick(*r["cout"])


def _args(g):
    return (g.stride[0], g.stride[1], g.padding[0], g.padding[2], g.dilation[0], g.dilation[1])


def _coef(C_, gpu):
    coef = torch.zeros(4, C_, device=gpu)
    coef[0].uniform_(0.3, 2.0)
    coef[1].normal_(0, 0.6)
    return coef


def _run_fwd(r, gpu, N, H, k, cin, cout, g):
    e = _ext()
    x = (torch.randn(N, H, H, cin) * 1.3 + 0.2).bfloat16().to(gpu)
    w = (torch.randn(cout, k, k, cin) / math.sqrt(k * k * cin)).bfloat16().to(gpu)
    if r["need"] & RF_FP8:
        from tensorflowdistributedlearning_amd.ops import fp8 as F8
        x8, sx = F8.quantize_e4m3(x)
        w8, sw = F8.quantize_e4m3(w)
        y = C.conv_fwd_fp8(x8, sx, w8, sw, g)
        ref = C.ref_conv_fwd(F8.dequantize(x8, sx).cpu(), F8.dequantize(w8, sw).cpu(), g)
        return y, ref, 1e-2
    stats = torch.zeros(2, cout, device=gpu)
    y = torch.empty(N, H, H, cout, device=gpu, dtype=torch.bfloat16)
    aff = None
    u = x
    if r["need"] & RF_AFF:
        aff = _coef(cin, gpu)
        u = B.bn_apply(x, aff, None, True)
    e.conv_fwd(x, w, y, None, stats, *_args(g), False, None, aff)
    torch.cuda.synchronize()
    ref = C.ref_conv_fwd(u.float().cpu(), w.float().cpu(), g)
    yb = y.float().cpu().reshape(-1, cout)
    if not e.deterministic():
        assert _rel(stats, torch.stack([yb.sum(0), (yb * yb).sum(0)])) < 1e-3
    return y, ref, 1e-2


def _run_dgrad(r, gpu, N, H, k, cin, cout, g):
    e = _ext()
    need = r["need"]
    w = (torch.randn(cout, k, k, cin) / math.sqrt(k * k * cout)).bfloat16().to(gpu)
    Ho, _ = g.out_hw(H, H, k, k)
    dy = torch.randn(N, Ho, Ho, cout).bfloat16().to(gpu)
    if need & RF_FP8:
        from tensorflowdistributedlearning_amd.ops import fp8 as F8
        dy8, sdy = F8.quantize_e5m2(dy)
        w8, sw = F8.quantize_e4m3(w)
        w8t = F8.transpose_weight(w8)
        wf8 = C.fp8_flip_weight(w8t) if need & RF_WFLIP else None
        dx = C.conv_dgrad_fp8(dy8, sdy, w8t, sw, (N, H, H, cin), g, w_flip=wf8)
        ref = C.ref_conv_dgrad(F8.dequantize_e5m2(dy8, sdy).cpu(), F8.dequantize(w8, sw).cpu(),
                               (N, H, H, cin), g)
        return dx, ref, 2e-2
    x = (torch.randn(N, H, H, cin) * 1.3 + 0.4).bfloat16().to(gpu)
    ref = C.ref_conv_dgrad(dy.float().cpu(), w.float().cpu(), x.shape, g)
    dx = torch.zeros_like(x)
    join = bool(need & RF_JOIN)
    if join:
        dx = torch.randn(N, H, H, cin).bfloat16().to(gpu)
        ref = ref + dx.float().cpu()
    bn_x = red = aff = None
    if need & RF_STATS:
        bn_x, red = x, torch.zeros(2, cin, device=gpu)
    if need & RF_AFF:
        aff = _coef(cin, gpu)
        mask = torch.empty(x.numel() // 8, device=gpu, dtype=torch.uint8)
        B.bn_apply(x, aff, None, True, mask=mask)
        ref = ref * B.unpack_relu_mask(mask.cpu(), cin).reshape(ref.shape)
    wf = None
    if need & RF_STRIDED:
        wf = C.flip_classes(w, g)
    elif need & RF_WFLIP:
        wf = torch.empty(cin, k, k, cout, device=gpu, dtype=torch.bfloat16)
        e.conv_flip_weight(w, wf)
    fused = e.conv_dgrad(dy, w, dx, *_args(g), join, None, None, bn_x, red, aff, wf)
    torch.cuda.synchronize()
    if need & RF_STATS and not e.deterministic():
        assert fused, f"{r['name']}: statistics row did not fuse the BN-backward sums"
        gf, xf = dx.float().cpu().reshape(-1, cin), x.float().cpu().reshape(-1, cin)
        assert _rel(red, torch.stack([gf.sum(0), (gf * xf).sum(0)])) < 1e-3
    return dx, ref, 1e-2


def _run_wgrad(r, gpu, N, H, k, cin, cout, g):
    e = _ext()
    x = torch.randn(N, H, H, cin).bfloat16().to(gpu)
    dy = torch.randn(N, H, H, cout).bfloat16().to(gpu)
    out = torch.empty(cout, k, k, cin, device=gpu)
    if r["need"] & RF_FP8:
        from tensorflowdistributedlearning_amd.ops import fp8 as F8
        x8, sx = F8.quantize_e4m3(x)
        dy8, sdy = F8.quantize_e5m2(dy)
        e.conv_wgrad_fp8(dy8, x8, out, sdy, sx, *_args(g), False)
        torch.cuda.synchronize()
        ref = C.ref_conv_wgrad(F8.dequantize_e5m2(dy8, sdy).cpu(), F8.dequantize(x8, sx).cpu(),
                               (cout, k, k, cin), g)
        return out, ref, 1e-3
    e.conv_wgrad(dy, x, out, None, *_args(g), False, None)
    torch.cuda.synchronize()
    ref = C.ref_conv_wgrad(dy.float().cpu(), x.float().cpu(), (cout, k, k, cin), g)
    return out, ref, 1e-3


@pytest.mark.parametrize("name", [r["name"] for r in ROWS])
def test_every_route_row_runs_and_matches_oracle(gpu, name):
    r = next(x for x in ROWS if x["name"] == name)
    op = OPS[r["op"]]
    k, cin, cout = _problem(r)
    p = (k - 1) // 2
    st = 2 if r["need"] & RF_STRIDED else 1
    g = C.ConvGeom((st, st), (p, p, p, p), (1, 1))
    N, H = 4, 14
    torch.manual_seed(zlib.crc32(name.encode()) % 1000)
    e = _ext()
    e.conv_route_force(op, name)
    try:
        run = {0: _run_fwd, 1: _run_dgrad, 2: _run_wgrad}[op]
        got, ref, tol = run(r, gpu, N, H, k, cin, cout, g)
        assert e.conv_last_route(op) == name
    finally:
        e.conv_route_force(op, "")
    assert got.shape == ref.shape
    assert _rel(got, ref) < tol, f"{name} (k{k} {cin}->{cout}): {_rel(got, ref):.2e}"


def test_forced_row_outside_its_window_raises(gpu):
    """A forced row that the problem does not fit is an error, not a silent fallback."""
    e = _ext()
    x = torch.randn(2, 14, 14, 64).bfloat16().to(gpu)
    w = torch.randn(64, 3, 3, 64).bfloat16().to(gpu)
    y = torch.empty(2, 14, 14, 64, device=gpu, dtype=torch.bfloat16)
    e.conv_route_force(0, "fwd.pc.wide3x3")  # needs >= 256 input channels
    try:
        with pytest.raises(RuntimeError, match="fwd.pc.wide3x3"):
            e.conv_fwd(x, w, y, None, None, 1, 1, 1, 1, 1, 1, False)
    finally:
        e.conv_route_force(0, "")


def test_route_cfg_override_runs_that_config(gpu):
    """conv_route_set(name, cfg=…) moves a row onto another instantiated tile config (the A/B
    knob); the result stays exact and the config is reported back by the table."""
    e = _ext()
    torch.manual_seed(5)
    x = torch.randn(8, 28, 28, 128).bfloat16().to(gpu)
    w = (torch.randn(256, 1, 1, 128) / 12).bfloat16().to(gpu)
    g = C.ConvGeom((1, 1), (0, 0, 0, 0), (1, 1))
    ref = C.ref_conv_fwd(x.float().cpu(), w.float().cpu(), g)
    try:
        for cfg in (0, 1, 2, 3, 4, 5):
            e.conv_route_set("fwd.glds.wide", cfg=cfg)
            assert next(r for r in e.conv_route_table() if r["name"] == "fwd.glds.wide")["cfg"] == cfg
            e.conv_route_force(0, "fwd.glds.wide")
            y = torch.empty(8, 28, 28, 256, device=gpu, dtype=torch.bfloat16)
            e.conv_fwd(x, w, y, None, None, 1, 1, 0, 0, 1, 1, False)
            torch.cuda.synchronize()
            assert e.conv_last_route(0) == "fwd.glds.wide"
            assert _rel(y, ref) < 1e-2, cfg
    finally:
        e.conv_route_force(0, "")
        e.conv_route_reset()


@pytest.mark.parametrize("N,H", [(2, 56), (3, 28), (2, 26), (3, 13)])
def test_resident_filter_conv_epilogues(gpu, N, H):
    """The resident-filter 3x3 64 -> 64 kernel (conv_halo.hip conv_rw_kernel; route rows
    fwd.halo.rw64 / dgrad.asfwd.rw64) with every epilogue it takes, against the fp32 oracle:
    forward with bias + fused BN sums (Σy, Σy²); input gradient (as the forward conv of dy with
    the flipped filter) with the ReLU bit mask, the residual join (dx += …) and the BN-backward
    sums (Σg, Σg·x) — on tile grids with ragged rows (H % 8) and a single column tile (H ≤ 30)."""
    e = _ext()
    torch.manual_seed(H)
    g = C.ConvGeom((1, 1), (1, 1, 1, 1), (1, 1))
    x = (torch.randn(N, H, H, 64) * 1.3 + 0.2).bfloat16().to(gpu)
    w = (torch.randn(64, 3, 3, 64) / 24).bfloat16().to(gpu)
    bias = torch.randn(64, device=gpu) * 0.1
    e.conv_route_force(0, "fwd.halo.rw64")
    try:
        stats = torch.zeros(2, 64, device=gpu)
        y = torch.empty(N, H, H, 64, device=gpu, dtype=torch.bfloat16)
        e.conv_fwd(x, w, y, bias, stats, *_args(g), False)
        torch.cuda.synchronize()
        assert e.conv_last_route(0) == "fwd.halo.rw64"
    finally:
        e.conv_route_force(0, "")
    ref = C.ref_conv_fwd(x.float().cpu(), w.float().cpu(), g) + bias.cpu()
    assert _rel(y, ref) < 1e-2
    yb = y.float().cpu().reshape(-1, 64)
    assert _rel(stats, torch.stack([yb.sum(0), (yb * yb).sum(0)])) < 1e-3

    # input gradient: mask of a BN output, join onto an existing dx, BN-backward sums against x
    dy = torch.randn(N, H, H, 64).bfloat16().to(gpu)
    coef = _coef(64, gpu)
    mask = torch.empty(x.numel() // 8, device=gpu, dtype=torch.uint8)
    B.bn_apply(x, coef, None, True, mask=mask)
    m = B.unpack_relu_mask(mask.cpu(), 64).reshape(N, H, H, 64)
    wf = torch.empty(64, 3, 3, 64, device=gpu, dtype=torch.bfloat16)
    e.conv_flip_weight(w, wf)
    base = C.ref_conv_dgrad(dy.float().cpu(), w.float().cpu(), x.shape, g)
    for join in (False, True):
        prev = torch.randn(N, H, H, 64).bfloat16().to(gpu) if join else None
        dx = prev.clone() if join else torch.empty_like(x)
        red = torch.zeros(2, 64, device=gpu)
        e.conv_route_force(1, "dgrad.asfwd.rw64")
        try:
            fused = e.conv_dgrad(dy, w, dx, *_args(g), join, mask, None, x, red, None, wf)
            torch.cuda.synchronize()
            assert e.conv_last_route(1) == "dgrad.asfwd.rw64"
        finally:
            e.conv_route_force(1, "")
        want = (base + (prev.float().cpu() if join else 0)) * m
        assert _rel(dx, want) < 1e-2, join
        if not e.deterministic():
            assert fused
            gf, xf = dx.float().cpu().reshape(-1, 64), x.float().cpu().reshape(-1, 64)
            assert _rel(red, torch.stack([gf.sum(0), (gf * xf).sum(0)])) < 1e-3


@pytest.mark.parametrize("k,cin,cout", [(1, 256, 64), (1, 1024, 256), (3, 128, 128)])
def test_wide_join_statistics_epilogue(gpu, k, cin, cout):
    """The residual join's last dgrad with the BN-backward sums on the 256×128 tiles (route row
    dgrad.asfwd.glds.join.wide: conv_common.h store_tile_bf16 loads its epilogue operands in two
    fragment-row halves): dx = (previous dx + dgrad)·[ReLU bit], (Σg, Σg·x) of the stored dx —
    the bottleneck conv1 joins of ResNet (1×1, C = 256 … 2048) and a 3×3 one."""
    e = _ext()
    torch.manual_seed(cin + k)
    N, H = 4, 14
    p = (k - 1) // 2
    g = C.ConvGeom((1, 1), (p, p, p, p), (1, 1))
    x = (torch.randn(N, H, H, cin) * 1.3 + 0.2).bfloat16().to(gpu)
    w = (torch.randn(cout, k, k, cin) / math.sqrt(k * k * cout)).bfloat16().to(gpu)
    dy = torch.randn(N, H, H, cout).bfloat16().to(gpu)
    coef = _coef(cin, gpu)
    mask = torch.empty(x.numel() // 8, device=gpu, dtype=torch.uint8)
    B.bn_apply(x, coef, None, True, mask=mask)
    m = B.unpack_relu_mask(mask.cpu(), cin).reshape(N, H, H, cin)
    wf = torch.empty(cin, k, k, cout, device=gpu, dtype=torch.bfloat16)
    e.conv_flip_weight(w, wf)
    prev = torch.randn(N, H, H, cin).bfloat16().to(gpu)
    dx = prev.clone()
    red = torch.zeros(2, cin, device=gpu)
    e.conv_route_force(1, "dgrad.asfwd.glds.join.wide")
    try:
        fused = e.conv_dgrad(dy, w, dx, *_args(g), True, mask, None, x, red, None, wf)
        torch.cuda.synchronize()
        assert e.conv_last_route(1) == "dgrad.asfwd.glds.join.wide"
    finally:
        e.conv_route_force(1, "")
    want = (C.ref_conv_dgrad(dy.float().cpu(), w.float().cpu(), x.shape, g)
            + prev.float().cpu()) * m
    assert _rel(dx, want) < 1e-2
    if not e.deterministic():
        assert fused
        gf, xf = dx.float().cpu().reshape(-1, cin), x.float().cpu().reshape(-1, cin)
        assert _rel(red, torch.stack([gf.sum(0), (gf * xf).sum(0)])) < 1e-3
