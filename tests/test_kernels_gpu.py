"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op
(SURVEY §7.5 "Kernel" tier).  Inputs are bf16; tolerances are relative to the reference's scale."""
import math

import pytest
import torch

from tensorflowdistributedlearning_amd.ops import conv as C
from tensorflowdistributedlearning_amd.ops import bn as B
from tensorflowdistributedlearning_amd.ops import pool as P
from tensorflowdistributedlearning_amd.ops import loss as L
from tensorflowdistributedlearning_amd.ops import optim as O
from tensorflowdistributedlearning_amd.ops import dwconv as D
from tensorflowdistributedlearning_amd.ops import upsample as U
from tensorflowdistributedlearning_amd.ops import metrics as Mt
from tensorflowdistributedlearning_amd.ops.common import ext

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


def bf(t, dev):
    return t.to(dev, torch.bfloat16)


# (N, H, W, C, K, R, S, stride, pad(t,b,l,r), dil)
CONV_SHAPES = [
    (2, 14, 14, 64, 64, 3, 3, 1, (1, 1, 1, 1), 1),      # resnet 3x3
    (2, 14, 14, 64, 256, 1, 1, 1, (0, 0, 0, 0), 1),     # 1x1 expand
    (2, 14, 14, 256, 128, 1, 1, 2, (0, 0, 0, 0), 1),    # 1x1 s2 downsample
    (2, 15, 15, 128, 128, 3, 3, 2, (1, 1, 1, 1), 1),    # 3x3 s2 odd
    (2, 16, 16, 64, 64, 3, 3, 2, (0, 1, 0, 1), 1),      # TF SAME asymmetric s2
    (2, 32, 32, 8, 64, 7, 7, 2, (3, 3, 3, 3), 1),       # stem (Cin padded to 8)
    (2, 13, 13, 64, 64, 3, 3, 1, (2, 2, 2, 2), 2),      # dilated r2
    (2, 13, 13, 64, 32, 3, 3, 1, (4, 4, 4, 4), 4),      # dilated r4
    (3, 1, 1, 200, 100, 1, 1, 1, (0, 0, 0, 0), 1),      # FC-shaped, ragged N
    (2, 13, 13, 258, 258, 3, 3, 1, (1, 1, 1, 1), 1),    # reference preset C=258 (generic path)
    (2, 9, 9, 40, 1, 3, 3, 1, (1, 1, 1, 1), 1),         # decoder 3x3 -> 1 channel
    (4, 7, 7, 512, 2048, 1, 1, 1, (0, 0, 0, 0), 1),     # layer4 expand
    (2, 13, 13, 24, 16, 3, 3, 2, (2, 2, 2, 2), 2),      # stride 2 + dilation 2 (masked dgrad)
    (1, 9, 9, 258, 40, 3, 3, 2, (1, 1, 1, 1), 1),       # C % 8 != 0 with parity classes
    (2, 11, 12, 16, 24, 1, 1, 2, (0, 0, 0, 0), 1),      # 1x1 s2 on odd/even sizes
    (2, 12, 12, 16, 16, 3, 3, 3, (1, 1, 1, 1), 1),      # stride 3 (9 parity classes)
    (64, 28, 28, 128, 128, 1, 1, 1, (0, 0, 0, 0), 1),   # multi-tile pipelining (tpb > 1)
    (16, 28, 28, 64, 64, 3, 3, 1, (1, 1, 1, 1), 1),     # LDS-DMA ring: many tiles per workgroup
    (8, 29, 27, 128, 192, 3, 3, 2, (1, 1, 1, 1), 1),    # ragged rows / cols, 4 parity classes
    (8, 20, 20, 40, 24, 3, 3, 1, (1, 1, 1, 1), 1),      # C, K % 64 != 0 (tap-crossing K-steps)
    (4, 33, 33, 256, 512, 1, 1, 2, (0, 0, 0, 0), 1),    # 1x1 s2, zero parity classes
    (2, 15, 15, 728, 200, 1, 1, 1, (0, 0, 0, 0), 1),    # 1x1, C and K % 64 != 0 (ragged FASTK)
    (2, 16, 16, 200, 328, 1, 1, 2, (0, 0, 0, 0), 1),    # 1x1 s2, ragged FASTK dgrad class
]

CONV_IMPLS = ["reg", "glds", "halo"]


@pytest.fixture(params=CONV_IMPLS)
def conv_impl(request, gpu):
    """Run a conv test with the register-staged kernels (0), the LDS-DMA kernels forced for
    every aligned problem (2), or the halo-tiled direct conv for every stride-1 problem it takes
    (conv_halo.hip; the others fall back to the default selection)."""
    ext().conv_set_glds_mode(0 if request.param == "reg" else 2 if request.param == "glds" else -1)
    ext().conv_set_halo_mode(2 if request.param == "halo" else 0)
    yield request.param
    ext().conv_set_glds_mode(-1)
    ext().conv_set_halo_mode(-1)


# (N, H, W, Cin, Cout, k, dil): halo tiles of one image, of several images (rows spanning image
# boundaries), dilation, multi-chunk Cin, ragged output-channel tiles, 64- and 128-wide tiles
HALO_SHAPES = [
    (4, 56, 56, 64, 64, 3, 1),      # ResNet layer1: 4-row tiles inside one image
    (6, 28, 28, 128, 128, 3, 1),    # 8-row tiles straddling images
    (8, 14, 14, 256, 256, 3, 1),    # 18-row tiles over up to 3 images
    (8, 7, 7, 512, 512, 3, 1),      # 28-row tiles = 4 images
    (4, 13, 13, 512, 256, 3, 2),    # DeepLab block3 dilation 2
    (3, 13, 13, 64, 32, 3, 4),      # dilation 4, Cout 32 (ragged 64-wide tile)
    (5, 17, 23, 192, 200, 3, 1),    # odd sizes, ragged Cout
    (2, 51, 51, 64, 128, 3, 1),     # DeepLab stem width 51
    (2, 20, 20, 128, 64, 5, 1),     # 5x5 filter
]


@pytest.mark.parametrize("shape", HALO_SHAPES)
def test_conv_halo_fwd_dgrad(gpu, shape):
    """Halo-tiled direct conv vs the fp32 oracle: forward with fused BN statistics, input
    gradient plain / accumulated (residual join) / ReLU-masked with BN-backward statistics."""
    from tensorflowdistributedlearning_amd.ops import bn as BN
    N, H, W, Cin, K, k, dil = shape
    p = dil * (k - 1) // 2
    g = C.ConvGeom((1, 1), (p, p, p, p), (dil, dil))
    torch.manual_seed(31)
    x = (torch.randn(N, H, W, Cin) * 1.3 + 0.2).bfloat16()
    w = (torch.randn(K, k, k, Cin) / math.sqrt(k * k * Cin)).bfloat16()
    ext().conv_set_halo_mode(2)
    try:
        ref = C.ref_conv_fwd(x.float(), w.float(), g)
        stats = torch.zeros(2, K, device=gpu)
        y = C.conv_fwd(x.to(gpu), w.to(gpu), g, stats=stats)
        assert rel_err(y, ref) < 2e-2
        yb = y.float().cpu().reshape(-1, K)
        assert rel_err(stats[0], yb.sum(0)) < 1e-3
        assert rel_err(stats[1], (yb * yb).sum(0)) < 1e-3
        dy = torch.randn(ref.shape).bfloat16()
        dx_ref = C.ref_conv_dgrad(dy.float(), w.float(), x.shape, g)
        dx = C.conv_dgrad(dy.to(gpu), w.to(gpu), x.shape, g)
        assert rel_err(dx, dx_ref) < 2e-2
        prev = torch.randn(N, H, W, Cin).bfloat16()
        out = prev.to(gpu)
        C.conv_dgrad(dy.to(gpu), w.to(gpu), x.shape, g, out=out, accumulate=True)
        assert rel_err(out, dx_ref + prev.float()) < 2e-2
        # masked dgrad with BN-backward statistics (the 3x3 conv2 of a bottleneck)
        xg = x.to(gpu)
        gam, bet = torch.rand(Cin, device=gpu) + 0.5, torch.randn(Cin, device=gpu) * 0.3
        coef = BN.bn_finalize(BN.bn_stats(xg), N * H * W, gam, bet, torch.zeros(Cin, device=gpu),
                              torch.ones(Cin, device=gpu), 0.9, 1e-3, True)
        mask = torch.empty(xg.numel() // 8, device=gpu, dtype=torch.uint8)
        BN.bn_apply(xg, coef, None, True, mask=mask)
        keep = BN.unpack_relu_mask(mask.cpu(), Cin).reshape(x.shape)
        dxm, red = C.conv_dgrad_bnstat(dy.to(gpu), w.to(gpu), x.shape, g, xg, mask=mask)
        assert rel_err(dxm, dx_ref * keep) < 2e-2
        assert (dxm.float().cpu()[~keep] == 0).all()
        if K % 64 == 0 and k * k <= 16:  # the halo dgrad takes it (K in 64-channel chunks)
            assert red is not None
        if red is not None:
            gf, xf = dxm.float().reshape(-1, Cin), xg.float().reshape(-1, Cin)
            assert rel_err(red, torch.stack([gf.sum(0), (gf * xf).sum(0)])) < 1e-4
        if k == 3:  # weight gradient (3x3 halo wgrad), fresh and accumulated
            dw_ref = C.ref_conv_wgrad(dy.float(), x.float(), w.shape, g)
            dw = C.conv_wgrad(dy.to(gpu), x.to(gpu), tuple(w.shape), g)
            assert rel_err(dw, dw_ref) < 1e-2
            out = dw.clone()
            C.conv_wgrad(dy.to(gpu), x.to(gpu), tuple(w.shape), g, out=out, accumulate=True)
            assert rel_err(out, 2 * dw_ref) < 1e-2
    finally:
        ext().conv_set_halo_mode(-1)


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_fwd_dgrad_wgrad(gpu, conv_impl, shape):
    N, H, W, Cin, K, R, S, st, pad, dil = shape
    g = C.ConvGeom((st, st), pad, (dil, dil))
    torch.manual_seed(0)
    x = torch.randn(N, H, W, Cin)
    w = torch.randn(K, R, S, Cin) / math.sqrt(R * S * Cin)
    xb, wb = x.bfloat16(), w.bfloat16()
    ref = C.ref_conv_fwd(xb.float(), wb.float(), g)
    stats = torch.zeros(2, K, device=gpu)
    y = C.conv_fwd(bf(x, gpu), bf(w, gpu), g, stats=stats)
    assert y.shape == ref.shape
    assert rel_err(y, ref) < 2e-2
    yb = y.float().cpu().reshape(-1, K)
    assert rel_err(stats[0], yb.sum(0)) < 1e-3
    assert rel_err(stats[1], (yb * yb).sum(0)) < 1e-3
    dy = torch.randn(ref.shape)
    dyb = dy.bfloat16()
    dx_ref = C.ref_conv_dgrad(dyb.float(), wb.float(), x.shape, g)
    dx = C.conv_dgrad(bf(dy, gpu), bf(w, gpu), x.shape, g)
    assert rel_err(dx, dx_ref) < 2e-2
    dw_ref = C.ref_conv_wgrad(dyb.float(), xb.float(), w.shape, g)
    dw = C.conv_wgrad(bf(dy, gpu), bf(x, gpu), tuple(w.shape), g)
    assert dw.dtype == torch.float32
    assert rel_err(dw, dw_ref) < 1e-2
    # accumulate mode + fused bias grad
    out = dw.clone()
    bgrad = torch.empty(K, device=gpu)
    C.conv_wgrad(bf(dy, gpu), bf(x, gpu), tuple(w.shape), g, out=out, accumulate=True,
                 bias_grad=bgrad)
    assert rel_err(out, 2 * dw_ref) < 1e-2
    assert rel_err(bgrad, dyb.float().reshape(-1, K).sum(0)) < 1e-2


def test_conv_bias_relu_epilogue(gpu, conv_impl):
    torch.manual_seed(1)
    g = C.ConvGeom((1, 1), (1, 1, 1, 1), (1, 1))
    x = torch.randn(2, 10, 10, 16).bfloat16()
    w = (torch.randn(24, 3, 3, 16) / 12).bfloat16()
    b = torch.randn(24)
    ref = torch.relu(C.ref_conv_fwd(x.float(), w.float(), g, b))
    y = C.conv_fwd(x.to(gpu), w.to(gpu), g, bias=b.to(gpu), relu=True)
    assert rel_err(y, ref) < 2e-2


def test_conv_large_resnet_shape(gpu):
    """A full-size ResNet-50 layer1 3x3 conv at batch 16 (many tiles, XCD remap, split-K wgrad)."""
    torch.manual_seed(2)
    g = C.ConvGeom((1, 1), (1, 1, 1, 1), (1, 1))
    x = torch.randn(16, 56, 56, 64).bfloat16()
    w = (torch.randn(64, 3, 3, 64) / 24).bfloat16()
    y = C.conv_fwd(x.to(gpu), w.to(gpu), g)
    ref = C.ref_conv_fwd(x.float(), w.float(), g)
    assert rel_err(y, ref) < 2e-2
    dy = torch.randn(ref.shape).bfloat16()
    dw = C.conv_wgrad(dy.to(gpu), x.to(gpu), tuple(w.shape), g)
    assert rel_err(dw, C.ref_conv_wgrad(dy.float(), x.float(), w.shape, g)) < 1e-2


@pytest.mark.parametrize("C_", [64, 258, 24])
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False), (2, False)])
def test_batchnorm(gpu, C_, relu, res):
    """relu=2: the backward kernels re-derive the ReLU mask from x·scale+shift (y not passed);
    checked against the mask-from-y reference."""
    torch.manual_seed(3)
    M = 2 * 9 * 11
    x = (torch.randn(2, 9, 11, C_) * 2 + 0.5).bfloat16()
    r = torch.randn(2, 9, 11, C_).bfloat16() if res else None
    gamma = torch.rand(C_) + 0.5
    beta = torch.randn(C_)
    rm, rv = torch.zeros(C_), torch.ones(C_)
    st_ref = B.bn_stats(x.float())
    coef_ref = B.bn_finalize(st_ref, M, gamma, beta, rm, rv, 0.9, 1e-3, True)
    y_ref = B.bn_apply(x.float(), coef_ref, None if r is None else r.float(), relu)
    xd = x.to(gpu)
    st = B.bn_stats(xd)
    assert rel_err(st, st_ref) < 1e-3
    rmd, rvd = torch.zeros(C_, device=gpu), torch.ones(C_, device=gpu)
    coef = B.bn_finalize(st, M, gamma.to(gpu), beta.to(gpu), rmd, rvd, 0.9, 1e-3, True)
    assert rel_err(coef, coef_ref) < 1e-3
    assert rel_err(rmd, rm) < 1e-3 and rel_err(rvd, rv) < 1e-3
    y = B.bn_apply(xd, coef, None if r is None else r.to(gpu), relu)
    assert rel_err(y, y_ref) < 2e-2
    dy = torch.randn(x.shape).bfloat16()
    ref_relu = bool(relu)
    y_dev = None if relu == 2 else y
    red_ref = B.bn_bwd_reduce(dy.float(), y.float().cpu(), x.float(), coef_ref, ref_relu)
    red = B.bn_bwd_reduce(dy.to(gpu), y_dev, xd, coef, relu)
    assert rel_err(red, red_ref) < 2e-2
    dx_ref, dres_ref = B.bn_bwd_apply(dy.float(), y.float().cpu(), x.float(), coef_ref, red_ref,
                                      gamma, M, ref_relu, res)
    dx, dres = B.bn_bwd_apply(dy.to(gpu), y_dev, xd, coef, red, gamma.to(gpu), M, relu, res)
    assert rel_err(dx, dx_ref) < 3e-2
    if res:
        assert rel_err(dres, dres_ref) < 1e-2


def test_batchnorm_autograd_matches_torch(gpu):
    """Whole BN+ReLU autograd Function vs torch.nn.functional.batch_norm (fp32)."""
    from tensorflowdistributedlearning_amd.models.layers import BatchNorm
    torch.manual_seed(4)
    bn = BatchNorm(32, decay=0.9, eps=1e-5).to(gpu)
    x = torch.randn(4, 6, 6, 32).bfloat16()
    xg = x.to(gpu).requires_grad_(True)
    y = bn(xg, relu=True)
    dy = torch.randn(y.shape).bfloat16()
    y.backward(dy.to(gpu))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    gr = torch.ones(32, requires_grad=True)
    br = torch.zeros(32, requires_grad=True)
    yr = torch.relu(torch.nn.functional.batch_norm(xr, None, None, gr, br, True, 0.1, 1e-5))
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert rel_err(y, yr.permute(0, 2, 3, 1)) < 2e-2
    assert rel_err(xg.grad, xr.grad.permute(0, 2, 3, 1)) < 3e-2
    assert rel_err(bn.gamma.grad, gr.grad) < 2e-2
    assert rel_err(bn.beta.grad, br.grad) < 2e-2


@pytest.mark.parametrize("k,s,pad,Cn", [(3, 2, (1, 1, 1, 1), 64), (3, 2, (0, 1, 0, 1), 16),
                                          (1, 2, (0, 0, 0, 0), 32), (3, 2, (1, 1, 1, 1), 5)])
def test_maxpool(gpu, k, s, pad, Cn):
    torch.manual_seed(5)
    x = torch.randn(2, 11, 12, Cn).bfloat16()
    xr = x.float().requires_grad_(True)
    yr = P.ref_max_pool(xr, k, s, pad)
    xg = x.to(gpu).requires_grad_(True)
    y = P.max_pool2d(xg, k, s, pad)
    assert rel_err(y, yr) < 1e-2
    dy = torch.randn(yr.shape).bfloat16()
    yr.backward(dy.float())
    y.backward(dy.to(gpu))
    assert rel_err(xg.grad, xr.grad) < 1e-2


def test_global_avg_pool(gpu):
    x = torch.randn(3, 7, 7, 64).bfloat16()
    xg = x.to(gpu).requires_grad_(True)
    y = P.global_avg_pool(xg)
    assert rel_err(y, x.float().mean((1, 2))) < 1e-2
    y.backward(torch.ones_like(y))
    assert rel_err(xg.grad, torch.full(x.shape, 1 / 49.0)) < 1e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("smooth", [0.0, 0.1])
def test_softmax_xent(gpu, dtype, smooth):
    torch.manual_seed(6)
    logits = (torch.randn(37, 1000) * 3).to(dtype)
    labels = torch.randint(0, 1000, (37,))
    l_ref, g_ref = L.ref_softmax_xent(logits.float(), labels, smooth)
    lg = logits.to(gpu).requires_grad_(True)
    loss = L.softmax_cross_entropy(lg, labels.to(gpu), smooth)
    assert abs(loss.item() - l_ref.item()) < 1e-3 * max(1, abs(l_ref.item()))
    loss.backward()
    assert rel_err(lg.grad, g_ref) < 2e-2


@pytest.mark.parametrize("P_", [101 * 101, 64, 1000, 16385, 256 * 256, 300 * 300])
def test_lovasz(gpu, P_):
    """One-workgroup LDS sort up to 16384 px, the multi-pass global bitonic path above (any
    input_shape beyond 128×128, as the reference's full top_k sort: core/losses.py:48-56)."""
    torch.manual_seed(7)
    Bn = 4
    logits = torch.randn(Bn, P_) * 2
    labels = (torch.rand(Bn, P_) > 0.6).float()
    labels[1] = 0.0  # empty mask image
    l_ref, g_ref = L.ref_lovasz_hinge(logits, labels)
    lg = logits.to(gpu).requires_grad_(True)
    loss = L.lovasz_hinge(lg, labels.to(gpu))
    assert abs(loss.item() - l_ref.item()) < 1e-4 * max(1.0, abs(l_ref.item()))
    loss.backward()
    assert rel_err(lg.grad, g_ref) < 1e-3


@pytest.mark.parametrize("P_", [101 * 101, 200 * 200])
def test_lovasz_nan_logit_stays_in_bounds(gpu, P_):
    """A NaN logit (diverged training) must give a non-finite loss, not an out-of-bounds
    gradient store: NaN errors sort first, padding entries never reach the first P positions.
    The other images' gradients are unaffected."""
    torch.manual_seed(10)
    logits = torch.randn(3, P_)
    labels = (torch.rand(3, P_) > 0.5).float()
    logits[2, 17] = float("nan")  # the last image: a stray padding index would write past grad
    lg = logits.to(gpu).requires_grad_(True)
    loss = L.lovasz_hinge(lg, labels.to(gpu))
    loss.backward()
    torch.cuda.synchronize()
    assert not math.isfinite(loss.item())
    _, g_ref = L.ref_lovasz_hinge(logits[:2], labels[:2])
    assert rel_err(lg.grad[:2] * 3 / 2, g_ref) < 1e-3  # (per-image mean over 3 vs 2 images)


@pytest.mark.parametrize("P_", [5000, 200 * 200])
def test_lovasz_ties(gpu, P_):
    """Heavily tied errors: the loss is order-independent within a tie (Σ over a tied run of
    e·Δjaccard telescopes), so it must match whatever tie order the reference sort picks."""
    torch.manual_seed(9)
    logits = torch.randint(-4, 5, (3, P_)).float() * 0.5
    labels = (torch.rand(3, P_) > 0.5).float()
    l_ref, _ = L.ref_lovasz_hinge(logits, labels)
    loss = L.lovasz_hinge(logits.to(gpu), labels.to(gpu))
    assert abs(loss.item() - l_ref.item()) < 1e-4 * max(1.0, abs(l_ref.item()))


def test_seg_metrics(gpu):
    torch.manual_seed(8)
    lab = (torch.rand(6, 101, 101, 1) > 0.5).float()
    pred = (torch.rand(6, 101, 101, 1) > 0.5).float()
    pred[0] = lab[0]
    lab[1] = 0
    pred[1] = 0
    for kaggle in (False, True):
        s_ref, a_ref = Mt.ref_seg_scores(lab, pred, kaggle)
        s, a = Mt.seg_scores(lab.to(gpu), pred.to(gpu), kaggle)
        assert rel_err(s, s_ref) < 1e-5 and rel_err(a, a_ref) < 1e-5


def test_sgd_adam(gpu):
    torch.manual_seed(9)
    n = 64 * 50
    p = torch.randn(n)
    g = torch.randn(n)
    flags = (torch.rand(n // 64) > 0.3).to(torch.uint8)
    m0 = torch.randn(n)
    pc, mc = p.clone(), m0.clone()
    O.sgd_momentum_(pc, g, mc, None, flags, 0.1, 0.9, 1e-4, 0.5, False)
    pg, mg = p.to(gpu), m0.to(gpu)
    lowp = torch.empty(n, dtype=torch.bfloat16, device=gpu)
    O.sgd_momentum_(pg, g.to(gpu), mg, lowp, flags.to(gpu), 0.1, 0.9, 1e-4, 0.5, False)
    assert rel_err(pg, pc) < 1e-6 and rel_err(mg, mc) < 1e-6
    assert rel_err(lowp, pc) < 1e-2
    v0 = torch.rand(n)
    pc, mc, vc = p.clone(), m0.clone(), v0.clone()
    O.adam_(pc, g, mc, vc, None, flags, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1.0)
    pg, mg, vg = p.to(gpu), m0.to(gpu), v0.to(gpu)
    O.adam_(pg, g.to(gpu), mg, vg, None, flags.to(gpu), 1e-3, 0.9, 0.999, 1e-8, 0.0, 1.0)
    assert rel_err(pg, pc) < 1e-6 and rel_err(vg, vc) < 1e-6


@pytest.mark.parametrize("Cn,rate,stride,relu", [(64, 2, 1, True), (1024, 8, 1, True),
                                                 (16, 1, 2, False), (1, 1, 1, False),
                                                 (728, 1, 1, False), (2048, 2, 1, True),
                                                 (128, 1, 2, True), (40, 1, 1, False)])
def test_depthwise(gpu, Cn, rate, stride, relu):
    torch.manual_seed(10)
    from tensorflowdistributedlearning_amd.models.layers import resolve_padding
    H = 13
    pad = resolve_padding("SAME", H, H, 3, 3, (stride, stride), (rate, rate))
    g = C.ConvGeom((stride, stride), pad, (rate, rate))
    x = torch.randn(2, H, H, Cn).bfloat16()
    w = (torch.randn(3, 3, Cn) * 0.3).bfloat16()
    b = torch.randn(Cn) * 0.1
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = D.ref_dw_fwd(xr, wr, g, br)
    if relu:
        yr = torch.relu(yr)
    wp = torch.nn.Parameter(w.float().to(gpu))
    wp._lowp = w.to(gpu)
    bp = torch.nn.Parameter(b.to(gpu))
    wp.grad = None
    xg = x.to(gpu).requires_grad_(True)
    y = D.depthwise_conv2d(xg, wp, bp, g, relu)
    assert rel_err(y, yr) < 2e-2
    dy = torch.randn(yr.shape).bfloat16()
    yr.backward(dy.float())
    y.backward(dy.to(gpu))
    assert rel_err(xg.grad, xr.grad) < 2e-2
    assert rel_err(wp.grad, wr.grad) < 2e-2
    assert rel_err(bp.grad, br.grad) < 2e-2


@pytest.mark.parametrize("Cn,rate,stride", [(64, 1, 1), (728, 1, 2), (128, 2, 1), (40, 1, 1),
                                            (1024, 1, 1)])
def test_depthwise_fused_input_relu(gpu, Cn, rate, stride):
    """relu_in: the kernels rectify x on load (fwd, wgrad) and mask dx by x > 0 (dgrad) — vs the
    fp32 reference of relu → depthwise conv (C = 40 takes the unfused fallback)."""
    torch.manual_seed(12)
    from tensorflowdistributedlearning_amd.models.layers import resolve_padding
    H = 17
    pad = resolve_padding("SAME", H, H, 3, 3, (stride, stride), (rate, rate))
    g = C.ConvGeom((stride, stride), pad, (rate, rate))
    x = torch.randn(2, H, H, Cn).bfloat16()
    w = (torch.randn(3, 3, Cn) * 0.3).bfloat16()
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = D.ref_dw_fwd(torch.relu(xr), wr, g)
    wp = torch.nn.Parameter(w.float().to(gpu))
    wp._lowp = w.to(gpu)
    xg = x.to(gpu).requires_grad_(True)
    y = D.depthwise_conv2d(xg, wp, None, g, False, relu_in=True)
    assert rel_err(y, yr) < 2e-2
    dy = torch.randn(yr.shape).bfloat16()
    yr.backward(dy.float())
    y.backward(dy.to(gpu))
    assert rel_err(xg.grad, xr.grad) < 2e-2
    assert rel_err(wp.grad, wr.grad) < 2e-2
    assert float(xg.grad.float()[xg.detach() <= 0].abs().max()) == 0.0


@pytest.mark.parametrize("hw,out", [((13, 13), (26, 26)), ((1, 1), (13, 13)), ((26, 26), (101, 101)),
                                    ((7, 5), (9, 12))])
def test_upsample(gpu, hw, out):
    torch.manual_seed(11)
    x = torch.randn(2, hw[0], hw[1], 16).bfloat16()
    xr = x.float().requires_grad_(True)
    yr = U.upsample(xr, out)
    xg = x.to(gpu).requires_grad_(True)
    y = U.upsample(xg, out)
    assert rel_err(y, yr) < 1e-2
    dy = torch.randn(yr.shape).bfloat16()
    yr.backward(dy.float())
    y.backward(dy.to(gpu))
    assert rel_err(xg.grad, xr.grad) < 2e-2


def test_native_extension_is_loaded(gpu):
    import sys
    from tensorflowdistributedlearning_amd import _native
    assert _native.available()
    assert any("_C" in (getattr(m, "__file__", "") or "") for m in list(sys.modules.values())
               if m is not None)


@pytest.mark.parametrize("shape", [(4, 14, 14, 256, 64, 1, 1, 1, (0, 0, 0, 0), 1),
                                   (4, 15, 15, 128, 256, 1, 1, 2, (0, 0, 0, 0), 1),
                                   (4, 14, 14, 64, 64, 3, 3, 1, (1, 1, 1, 1), 1),
                                   (8, 28, 28, 128, 128, 3, 3, 2, (1, 1, 1, 1), 1)])
def test_conv_dgrad_accumulate(gpu, conv_impl, shape):
    """Residual-gradient join: dgrad epilogue adds into an existing dx (zero parity classes of a
    strided 1x1 keep the existing values)."""
    N, H, W, Cin, K, R, S, st, pad, dil = shape
    g = C.ConvGeom((st, st), pad, (dil, dil))
    torch.manual_seed(5)
    w = (torch.randn(K, R, S, Cin) / math.sqrt(R * S * Cin)).bfloat16()
    Ho, Wo = g.out_hw(H, W, R, S)
    dy = torch.randn(N, Ho, Wo, K).bfloat16()
    prev = torch.randn(N, H, W, Cin).bfloat16()
    ref = prev.float() + C.ref_conv_dgrad(dy.float(), w.float(), (N, H, W, Cin), g)
    out = prev.to(gpu)
    C.conv_dgrad(dy.to(gpu), w.to(gpu), (N, H, W, Cin), g, out=out, accumulate=True)
    assert rel_err(out, ref) < 2e-2


@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("shape", [(4, 14, 14, 256, 64, 1, 1, 1, (0, 0, 0, 0), 1),
                                   (4, 15, 15, 128, 256, 1, 1, 2, (0, 0, 0, 0), 1),
                                   (8, 28, 28, 128, 128, 3, 3, 2, (1, 1, 1, 1), 1),
                                   (64, 28, 28, 128, 128, 1, 1, 1, (0, 0, 0, 0), 1)])
def test_conv_dgrad_relu_mask(gpu, conv_impl, shape, accumulate):
    """Pre-masked join (ops/gradjoin.py): the dgrad epilogue multiplies what it writes by a
    1-bit-per-element ReLU mask, dx = ([dx +] dgrad)·[bit]; pixels a strided dgrad does not
    touch keep their previous value (accumulate) or are zero (overwrite) — vs the CPU oracle."""
    from tensorflowdistributedlearning_amd.ops import bn as BN
    N, H, W, Cin, K, R, S, st, pad, dil = shape
    g = C.ConvGeom((st, st), pad, (dil, dil))
    torch.manual_seed(9)
    w = (torch.randn(K, R, S, Cin) / math.sqrt(R * S * Cin)).bfloat16()
    Ho, Wo = g.out_hw(H, W, R, S)
    dy = torch.randn(N, Ho, Wo, K).bfloat16()
    prev = torch.randn(N, H, W, Cin).bfloat16()
    keep = torch.rand(N, H, W, Cin) > 0.4
    bits = keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)
    mask = bits.sum(1).to(torch.uint8)
    assert torch.equal(BN.unpack_relu_mask(mask, Cin).reshape(keep.shape), keep)
    ref = C.ref_conv_dgrad(dy.float(), w.float(), (N, H, W, Cin), g)
    if accumulate:
        ref = ref + prev.float()
        keep = keep | ~C._dgrad_touched(w.shape, (N, H, W, Cin), g)  # untouched: prev kept
    ref = ref * keep
    cpu = C.conv_dgrad(dy.float(), w.float(), (N, H, W, Cin), g, mask=mask,
                       out=prev.float().clone() if accumulate else None, accumulate=accumulate)
    assert rel_err(cpu, ref) < 1e-5
    out = prev.to(gpu) if accumulate else None
    dx = C.conv_dgrad(dy.to(gpu), w.to(gpu), (N, H, W, Cin), g, out=out, accumulate=accumulate,
                      mask=mask.to(gpu))
    assert rel_err(dx, ref) < 2e-2
    assert (dx.float().cpu()[~keep] == 0).all()  # masked elements exactly zero


@pytest.mark.parametrize("shape", [(8, 28, 28, 128, 256, 1, 1, False),   # 1x1, 8-wave 128x128
                                   (8, 28, 28, 64, 256, 1, 1, False),    # 64-wide dx (cfg 4)
                                   (8, 14, 14, 128, 128, 3, 1, False),   # 3x3
                                   (8, 28, 28, 256, 64, 1, 1, True),     # join accumulate
                                   (8, 30, 30, 192, 128, 1, 1, False),   # ragged column tiles
                                   (8, 28, 28, 128, 128, 3, 2, False),   # strided: 4 classes
                                   (8, 28, 28, 128, 256, 1, 2, False),   # 1x1/s2: zero classes
                                   (8, 28, 28, 256, 128, 1, 2, True)])   # strided join: no
def test_conv_dgrad_bnstat(gpu, shape):
    """BN-backward statistics fused into the LDS-DMA dgrad epilogue (ops/gradjoin.py): dx is
    bit-identical to the plain masked dgrad, and (Σg, Σg·x) of the stored dx match an fp32
    reduction; strided dgrads report no statistics.  bn_bwd_apply(red_raw=True) on them equals
    the reduce-pass path."""
    N, H, W, Cin, K, k, st, join = shape
    p = (k - 1) // 2
    g = C.ConvGeom((st, st), (p, p, p, p), (1, 1))
    torch.manual_seed(21)
    w = (torch.randn(K, k, k, Cin) / math.sqrt(k * k * Cin)).bfloat16().to(gpu)
    Ho, Wo = g.out_hw(H, W, k, k)
    dy = torch.randn(N, Ho, Wo, K).bfloat16().to(gpu)
    x = (torch.randn(N, H, W, Cin) * 1.3 + 0.4).bfloat16().to(gpu)
    gam, bet = torch.rand(Cin, device=gpu) + 0.5, torch.randn(Cin, device=gpu) * 0.3
    M = N * H * W
    coef = B.bn_finalize(B.bn_stats(x), M, gam, bet, torch.zeros(Cin, device=gpu),
                         torch.ones(Cin, device=gpu), 0.9, 1e-3, True)
    mask = torch.empty(x.numel() // 8, device=gpu, dtype=torch.uint8)
    B.bn_apply(x, coef, None, True, mask=mask)
    prev = torch.randn(N, H, W, Cin).bfloat16().to(gpu) if join else None
    ext().conv_set_glds_mode(2)  # the LDS-DMA kernel for these small problems too
    try:
        ref = C.conv_dgrad(dy, w, x.shape, g, mask=mask,
                           out=prev.clone() if join else None, accumulate=join)
        dx, red = C.conv_dgrad_bnstat(dy, w, x.shape, g, x, mask=mask,
                                      out=prev.clone() if join else None, accumulate=join)
    finally:
        ext().conv_set_glds_mode(-1)
    assert torch.equal(dx, ref)
    if st != 1 and join:
        assert red is None
        return
    assert red is not None
    gf, xf = dx.float().reshape(-1, Cin), x.float().reshape(-1, Cin)
    want = torch.stack([gf.sum(0), (gf * xf).sum(0)])
    assert rel_err(red, want) < 1e-4
    d0, _ = B.bn_bwd_apply(dx, None, x, coef, B.bn_bwd_reduce(dx, None, x, coef, 0), gam, M, 0,
                           False)
    d1, _ = B.bn_bwd_apply(dx, None, x, coef, red, gam, M, 0, False, red_raw=True)
    assert rel_err(d1, d0) < 1e-2


def test_fp8_quantize_matches_cpu(gpu):
    from tensorflowdistributedlearning_amd.ops import fp8 as F8
    torch.manual_seed(12)
    x = (torch.randn(4, 7, 9, 32) * 3).bfloat16()
    y8c, sc = F8.quantize_e4m3(x)
    y8g, sg = F8.quantize_e4m3(x.to(gpu))
    assert abs(float(sg) - float(sc)) / float(sc) < 1e-6
    diff = (y8g.cpu().view(torch.uint8).int() - y8c.view(torch.uint8).int()).abs()
    assert (diff > 0).float().mean() < 1e-3 and diff.max() <= 1  # RNE ties at most one ulp apart
    back = F8.dequantize(y8g, sg).cpu()
    assert rel_err(back, x.float()) < 0.07  # e4m3: 3 mantissa bits


@pytest.mark.parametrize("res", [False, True])
def test_bn_apply_fp8_side_output(gpu, res):
    """Delayed scaling: call 1 only measures |y|max; call 2 writes e4m3(y / (amax_1/448)) and the
    scale; the ring rotates (prev, out, cleared) without a memset launch."""
    from tensorflowdistributedlearning_amd.ops import bn as B, fp8 as F8
    torch.manual_seed(21)
    Cc = 64
    x = torch.randn(64, 15, 17, Cc, device=gpu).bfloat16()  # > AMAX_SPREAD workgroups
    r = torch.randn(64, 15, 17, Cc, device=gpu).bfloat16() if res else None
    coef = torch.stack([torch.rand(Cc) + 0.5, torch.randn(Cc) * 0.1,
                        torch.zeros(Cc), torch.ones(Cc)]).to(gpu)
    ring = torch.zeros(3, F8.AMAX_SLOT, device=gpu)
    ring[2] = 123.0  # stale value: must be cleared by call 1
    slot = lambda k: float(ring[k].view(16, 64)[:, 0].max())
    y1 = B.bn_apply(x, coef, r, True, (ring, 0, torch.zeros(1, device=gpu), False))
    assert not hasattr(y1, "_tdl_fp8")
    amax1 = float(y1.float().abs().max())
    assert slot(1) == amax1 and slot(2) == 0.0
    x2 = x * 0.5
    y2 = B.bn_apply(x2, coef, r, True, (ring, 1, torch.zeros(1, device=gpu), True))
    y8, sc = y2._tdl_fp8
    assert abs(float(sc) - amax1 / 448) < 1e-7 * amax1
    assert slot(2) == float(y2.float().abs().max()) and slot(0) == 0.0
    back = F8.dequantize(y8, sc).cpu()
    assert rel_err(back, y2.float().cpu()) < 0.07
    assert torch.equal(y2, B.bn_apply(x2, coef, r, True))  # bf16 output unchanged


def test_fp8_delayed_scaler(gpu):
    """First call exact (primed), later calls use the previous call's amax and saturate.  The
    scale lives in one device slot per scaler (graph-capturable; its consumers run before the
    next call), so each value is read right after its call."""
    from tensorflowdistributedlearning_amd.ops import fp8 as F8
    torch.manual_seed(22)
    sc = F8.DelayedScaler()
    x1 = torch.randn(1000, 64, device=gpu).bfloat16()
    y1, s1 = sc.quantize(x1)
    v1 = float(s1)
    ref1, r1 = F8.quantize_e4m3(x1.cpu())
    assert abs(v1 - float(r1)) <= 1e-6 * float(r1)
    x2 = x1 * 2
    y2, s2 = sc.quantize(x2)
    v2 = float(s2)
    assert abs(v2 - v1) <= 1e-7  # scale from call 1
    d2 = F8.dequantize(y2, s2).cpu()
    assert float(d2.abs().max()) <= v1 * 448 * (1 + 1e-6)  # saturated at the old amax
    y3, s3 = sc.quantize(x2)
    assert abs(float(s3) - 2 * v1) <= 1e-6 * float(s3)  # call 2 measured 2x


@pytest.mark.parametrize("shape", [(8, 14, 14, 128, 256, 3, 3, 1, 1),     # C % 128 == 0: tap per step
                                   (8, 14, 14, 64, 128, 3, 3, 1, 1),      # 2 taps per 128-deep step
                                   (4, 15, 15, 256, 64, 1, 1, 2, 0),      # 1x1 s2, 256x64 config
                                   (16, 7, 7, 512, 512, 3, 3, 1, 1),
                                   (2, 9, 11, 48, 40, 3, 3, 2, 1)])       # ragged everything
def test_conv_fwd_fp8(gpu, shape):
    from tensorflowdistributedlearning_amd.ops import fp8 as F8
    N, H, W, Cin, K, R, S, st, p = shape
    g = C.ConvGeom((st, st), (p, p, p, p), (1, 1))
    torch.manual_seed(13)
    x = torch.randn(N, H, W, Cin).bfloat16()
    w = (torch.randn(K, R, S, Cin) / math.sqrt(R * S * Cin)).bfloat16()
    x8, sx = F8.quantize_e4m3(x.to(gpu))
    w8, sw = F8.quantize_e4m3(w.to(gpu))
    ref = C.ref_conv_fwd(F8.dequantize(x8, sx).cpu(), F8.dequantize(w8, sw).cpu(), g)
    stats = torch.zeros(2, K, device=gpu)
    y = C.conv_fwd_fp8(x8, sx, w8, sw, g, stats=stats)
    assert y.dtype == torch.bfloat16 and y.shape == ref.shape
    assert rel_err(y, ref) < 1e-2
    yb = y.float().cpu().reshape(-1, K)
    assert rel_err(stats[0], yb.sum(0)) < 1e-3
    # fp8 vs the bf16 conv of the unquantised data: quantisation error only
    assert rel_err(y, C.ref_conv_fwd(x.float(), w.float(), g)) < 0.08


@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("shape", [(4, 14, 14, 64, 128, 3, 3, 1, 1),     # 3x3, Ng 64 (256x64 tiles)
                                   (4, 15, 15, 256, 128, 1, 1, 2, 0),   # 1x1/s2: empty classes
                                   (8, 28, 28, 128, 256, 3, 3, 2, 1),   # 3x3/s2: 4 parity classes
                                   (16, 14, 14, 512, 256, 1, 1, 1, 0)])  # 1x1, many tiles
def test_conv_dgrad_fp8(gpu, shape, accumulate):
    """fp8 dgrad (e5m2 dy × e4m3 W^T on the f8f6f4 MFMA, LDS-DMA kernel) vs the fp32 dgrad of the
    same dequantised operands; with accumulate, the join's dx += … plus the ReLU bit mask."""
    from tensorflowdistributedlearning_amd.ops import fp8 as F8, bn as BN
    N, H, W, Cin, K, R, S, st, p = shape
    g = C.ConvGeom((st, st), (p, p, p, p), (1, 1))
    torch.manual_seed(17)
    Ho, Wo = g.out_hw(H, W, R, S)
    dy = torch.randn(N, Ho, Wo, K).bfloat16()
    w = (torch.randn(K, R, S, Cin) / math.sqrt(R * S * K)).bfloat16()
    dy8, sdy = F8.quantize_e5m2(dy.to(gpu))
    w8, sw = F8.quantize_e4m3(w.to(gpu))
    w8t = F8.transpose_weight(w8)
    assert w8t.shape == (R, S, Cin, K)
    ref = C.ref_conv_dgrad(F8.dequantize_e5m2(dy8, sdy).cpu(), F8.dequantize(w8, sw).cpu(),
                           (N, H, W, Cin), g)
    prev = torch.randn(N, H, W, Cin).bfloat16()
    mask = None
    if accumulate:
        keep = torch.rand(N, H, W, Cin) > 0.3
        bits = keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)
        mask = bits.sum(1).to(torch.uint8)
        touched = C._dgrad_touched(w.shape, (N, H, W, Cin), g)
        ref = (ref + prev.float()) * (keep | ~touched)
    out = prev.to(gpu) if accumulate else None
    dx = C.conv_dgrad_fp8(dy8, sdy, w8t, sw, (N, H, W, Cin), g, out=out, accumulate=accumulate,
                          mask=None if mask is None else mask.to(gpu))
    assert dx.dtype == torch.bfloat16 and dx.shape == ref.shape
    assert rel_err(dx, ref) < 2e-2
    if not accumulate:  # vs the bf16 dgrad of the unquantised data: quantisation error only
        assert rel_err(dx, C.ref_conv_dgrad(dy.float(), w.float(), (N, H, W, Cin), g)) < 0.15


@pytest.mark.parametrize("shape", [(4, 14, 14, 64, 128, 3, 3, 1, 1), (4, 14, 14, 256, 256, 1, 1, 2, 0),
                                   (2, 9, 9, 128, 128, 3, 3, 2, 1)])
@pytest.mark.parametrize("masked,join", [(False, False), (True, False), (True, True)])
def test_conv_dgrad_fp8_bnstat(gpu, shape, masked, join):
    """fp8 dgrad with the BN-backward statistics in its epilogue: dx as the plain fp8 dgrad, and
    (Σg, Σg·x) of the stored (masked) dx against the same sums computed from it; ``join``: the
    residual join's dx += … (stride 1; the strided shapes then take the BN's own reduce)."""
    from tensorflowdistributedlearning_amd.ops import fp8 as F8
    from tensorflowdistributedlearning_amd.ops.common import ext
    if ext().deterministic():
        pytest.skip("deterministic mode: no fused epilogue sums")
    N, H, W, Cin, K, R, S, st, p = shape
    g = C.ConvGeom((st, st), (p, p, p, p), (1, 1))
    torch.manual_seed(23)
    Ho, Wo = g.out_hw(H, W, R, S)
    dy8, sdy = F8.quantize_e5m2(torch.randn(N, Ho, Wo, K).bfloat16().to(gpu))
    w8, sw = F8.quantize_e4m3((torch.randn(K, R, S, Cin) / math.sqrt(R * S * K)).bfloat16().to(gpu))
    w8t = F8.transpose_weight(w8)
    bn_x = (torch.randn(N, H, W, Cin) * 1.5 + 0.3).bfloat16().to(gpu)
    mask = None
    if masked:
        keep = torch.rand(N, H, W, Cin) > 0.4
        bits = keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)
        mask = bits.sum(1).to(torch.uint8).to(gpu)
    prev = torch.randn(N, H, W, Cin).bfloat16().to(gpu) if join else None
    plain = C.conv_dgrad_fp8(dy8, sdy, w8t, sw, (N, H, W, Cin), g, mask=mask,
                             out=None if prev is None else prev.clone(), accumulate=join)
    dx, red = C.conv_dgrad_fp8(dy8, sdy, w8t, sw, (N, H, W, Cin), g, mask=mask, bn_x=bn_x,
                               out=None if prev is None else prev.clone(), accumulate=join)
    if join and st > 1:
        assert red is None  # strided joins: not fused (pixels of tap-less classes stay unmasked)
        return
    assert red is not None, "fp8 dgrad did not fuse the statistics"
    assert torch.equal(dx, plain)
    gf, xf = dx.float().cpu().reshape(-1, Cin), bn_x.float().cpu().reshape(-1, Cin)
    want = torch.stack([gf.sum(0), (gf * xf).sum(0)])
    assert rel_err(red.cpu(), want) < 1e-3


@pytest.mark.parametrize("shape", [(4, 14, 14, 256, 128, 1, 1, 1, 0), (2, 14, 14, 64, 256, 3, 3, 1, 1)])
@pytest.mark.parametrize("mode", ["plain", "stats", "join"])
def test_conv_dgrad_fp8_as_forward(gpu, shape, mode):
    """The fp8 dgrad as the forward fp8 conv of e5m2 dy with the e4m3 flipped filter (route row
    dgrad.asfwd.fp8) against the fp8 DGRAD kernel on the same operands: dx (with the ReLU mask,
    and the join's accumulate), and the fused BN-backward sums."""
    from tensorflowdistributedlearning_amd.ops import fp8 as F8
    from tensorflowdistributedlearning_amd.ops.common import ext
    N, H, W, Cin, K, R, S, st, p = shape
    g = C.ConvGeom((st, st), (p, p, p, p), (1, 1))
    torch.manual_seed(31)
    dy8, sdy = F8.quantize_e5m2(torch.randn(N, H, W, K).bfloat16().to(gpu))
    w8, sw = F8.quantize_e4m3((torch.randn(K, R, S, Cin) / math.sqrt(R * S * K)).bfloat16().to(gpu))
    w8t = F8.transpose_weight(w8)
    wf8 = C.fp8_flip_weight(w8t)
    keep = torch.rand(N, H, W, Cin) > 0.4
    bits = keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)
    mask = bits.sum(1).to(torch.uint8).to(gpu)
    bn_x = (torch.randn(N, H, W, Cin) + 0.3).bfloat16().to(gpu) if mode != "plain" else None
    prev = torch.randn(N, H, W, Cin).bfloat16().to(gpu) if mode == "join" else None
    kw = dict(mask=mask, out=None if prev is None else prev.clone(), accumulate=mode == "join")
    ref = C.conv_dgrad_fp8(dy8, sdy, w8t, sw, (N, H, W, Cin), g, **kw)
    kw = dict(mask=mask, out=None if prev is None else prev.clone(), accumulate=mode == "join")
    ext().conv_route_force(1, "dgrad.asfwd.fp8")
    try:
        got = C.conv_dgrad_fp8(dy8, sdy, w8t, sw, (N, H, W, Cin), g, bn_x=bn_x, w_flip=wf8, **kw)
        assert ext().conv_last_route(1) == "dgrad.asfwd.fp8"
    finally:
        ext().conv_route_force(1, "")
    dx, red = got if bn_x is not None else (got, None)
    assert rel_err(dx, ref) < 1e-2
    if bn_x is not None and not ext().deterministic():
        assert red is not None
        gf, xf = dx.float().cpu().reshape(-1, Cin), bn_x.float().cpu().reshape(-1, Cin)
        assert rel_err(red.cpu(), torch.stack([gf.sum(0), (gf * xf).sum(0)])) < 1e-3


@pytest.mark.parametrize("k,s,p", [(3, 2, 1), (1, 2, 0), (3, 3, 1), (5, 2, 2), (2, 2, 0)])
def test_flip_classes_native_matches_reference(gpu, k, s, p):
    """ops/conv.flip_classes on the GPU (one conv_flip_classes launch) equals the ATen slice /
    flip / permute / cat form bit for bit, classes a-major, empty classes skipped."""
    torch.manual_seed(37)
    w = torch.randn(48, k, k, 24).bfloat16()
    g = C.ConvGeom((s, s), (p, p, p, p), (1, 1))
    ref = C.flip_classes(w, g)  # CPU: the reference form
    got = C.flip_classes(w.to(gpu), g)
    assert got.shape == ref.shape and torch.equal(got.cpu(), ref)


def test_fp8_e5m2_quantize_and_transpose(gpu):
    from tensorflowdistributedlearning_amd.ops import fp8 as F8
    torch.manual_seed(19)
    x = (torch.randn(3, 5, 7, 32) * 40).bfloat16()
    y8, s = F8.quantize_e5m2(x.to(gpu))
    yc, sc = F8.quantize_e5m2(x)
    torch.testing.assert_close(s.cpu(), sc, rtol=1e-6, atol=0)
    deq = F8.dequantize_e5m2(y8, s).cpu()
    assert rel_err(deq, yc.float() * sc) < 1e-6     # same e5m2 codes as torch's RNE conversion
    assert rel_err(deq, x.float()) < 0.13           # 2 mantissa bits
    w8, _ = F8.quantize_e4m3(torch.randn(128, 3, 3, 64, device=gpu).bfloat16())
    torch.testing.assert_close(F8.transpose_weight(w8).view(torch.uint8).cpu(),
                               w8.view(torch.uint8).cpu().permute(1, 2, 3, 0).contiguous())


def test_bn_bwd_apply_e5m2_side_output(gpu):
    """BN backward apply's e5m2 copy of dx (delayed scaling: the first call only measures, the
    second quantises with the first call's |dx|max)."""
    from tensorflowdistributedlearning_amd.ops import fp8 as F8
    torch.manual_seed(21)
    M, Cc = 2 * 9 * 11, 128
    x = (torch.randn(2, 9, 11, Cc) * 2 + 0.5).bfloat16().to(gpu)
    dy = torch.randn(2, 9, 11, Cc).bfloat16().to(gpu)
    st = B.bn_stats(x)
    coef = B.bn_finalize(st, M, torch.ones(Cc, device=gpu), torch.zeros(Cc, device=gpu),
                         torch.zeros(Cc, device=gpu), torch.ones(Cc, device=gpu), 0.9, 1e-3, True)
    red = B.bn_bwd_reduce(dy, None, x, coef, 2)
    sc = F8.DelayedScaler()
    dx0, _ = B.bn_bwd_apply(dy, None, x, coef, red, torch.ones(Cc, device=gpu), M, 2, False,
                            fp8=sc.bn_args(x))
    assert getattr(dx0, "_tdl_fp8", None) is None       # first call: measure only
    dx1, _ = B.bn_bwd_apply(dy, None, x, coef, red, torch.ones(Cc, device=gpu), M, 2, False,
                            fp8=sc.bn_args(x))
    dx8, s = dx1._tdl_fp8
    assert dx8.dtype == torch.float8_e5m2
    margin = ext().fp8_policy()[1]  # e5m2 headroom over the previous |dx|max (default 16×)
    torch.testing.assert_close(float(s), margin * float(dx0.float().abs().max()) / F8.E5M2_MAX,
                               rtol=1e-6, atol=0)
    assert rel_err(F8.dequantize_e5m2(dx8, s), dx1) < 0.13


def test_fp8_flat_weights_one_launch(gpu):
    """All fp8 weights of a flat buffer re-quantised by one launch per parameter version; the
    first version is exact (primed), later versions use the previous amax."""
    from tensorflowdistributedlearning_amd.ops import fp8 as F8
    from tensorflowdistributedlearning_amd.models.params import FlatParams, version, bump_version
    torch.manual_seed(23)
    mod = torch.nn.Module()
    mod.a = torch.nn.Parameter(torch.randn(64, 3, 3, 32))
    mod.b = torch.nn.Parameter(torch.randn(40000, 16) * 5)  # > one chunk
    mod.c = torch.nn.Parameter(torch.randn(7))               # not fp8
    fp = FlatParams(mod, gpu)
    fw = F8.flat_weights_for(mod.a)
    assert fw.get(mod.a, version()) is None and fw.get(mod.b, version()) is None
    bump_version()
    for p in (mod.a, mod.b):
        w8, s = fw.get(p, version())
        ref8, rs = F8.quantize_e4m3(p._lowp.cpu())
        assert abs(float(s) - float(rs)) <= 1e-6 * float(rs)
        assert w8.shape == p.shape
        assert rel_err(F8.dequantize(w8, s).cpu(), p._lowp.float().cpu()) < 0.07
    with torch.no_grad():
        mod.b.mul_(2)
    fp.sync_lowp()
    w8, s = fw.get(mod.b, version())
    w8b, sb = fw.get(mod.b, version())  # same version: no relaunch, same views
    assert w8b.data_ptr() == w8.data_ptr()
    amax_old = float(mod.b._lowp.float().abs().max()) / 2  # bf16 copy: exact halving
    assert abs(float(s) - amax_old / 448) <= 1e-5 * float(s)  # delayed: previous version's amax
    fp.sync_lowp()
    w8, s = fw.get(mod.b, version())
    assert abs(float(s) - 2 * amax_old / 448) <= 1e-5 * float(s)


@pytest.mark.parametrize("C_", [64, 264, 2048])
def test_batchnorm_bitmask_relu(gpu, C_):
    """relu mode 3 (residual BN): bn_apply writes the ReLU mask as one bit per element and both
    backward kernels read it instead of y — same results as the mask-from-y mode 1."""
    torch.manual_seed(8)
    M = 2 * 9 * 11
    x = (torch.randn(2, 9, 11, C_) * 2 + 0.5).bfloat16().to(gpu)
    r = torch.randn(2, 9, 11, C_).bfloat16().to(gpu)
    gamma = (torch.rand(C_) + 0.5).to(gpu)
    beta = torch.randn(C_).to(gpu)
    st = B.bn_stats(x)
    coef = B.bn_finalize(st, M, gamma, beta, torch.zeros(C_, device=gpu),
                         torch.ones(C_, device=gpu), 0.9, 1e-3, True)
    mask = torch.empty(x.numel() // 8, device=gpu, dtype=torch.uint8)
    y = B.bn_apply(x, coef, r, True, mask=mask)
    assert torch.equal(y, B.bn_apply(x, coef, r, True))
    assert torch.equal(B.unpack_relu_mask(mask, C_), y.float().reshape(-1, C_) > 0)
    dy = torch.randn(x.shape).bfloat16().to(gpu)
    red1 = B.bn_bwd_reduce(dy, y, x, coef, 1)
    red3 = B.bn_bwd_reduce(dy, mask, x, coef, 3)
    torch.testing.assert_close(red3, red1, rtol=1e-4, atol=1e-4)
    dx1, dr1 = B.bn_bwd_apply(dy, y, x, coef, red1, gamma, M, 1, True)
    dx3, dr3 = B.bn_bwd_apply(dy, mask, x, coef, red1, gamma, M, 3, True)
    assert torch.equal(dx1, dx3) and torch.equal(dr1, dr3)


@pytest.mark.parametrize("shape", [(4, 14, 14, 64, 128, 3, 1, (1, 1, 1, 1)),
                                   (8, 16, 16, 128, 64, 1, 2, (0, 0, 0, 0))])
def test_conv_dgrad_transposed_weights(gpu, shape):
    """conv_dgrad(w_t=[R,S,C,K] copy): the LDS-DMA kernel's K-contiguous B-operand variant gives
    the same bits as the transposed-LDS-read path (same products, same order)."""
    N, H, _, Cin, K, k, s, pad = shape
    g = C.ConvGeom((s, s), pad, (1, 1))
    torch.manual_seed(5)
    w = (torch.randn(K, k, k, Cin) * 0.05).bfloat16().to(gpu)
    Ho, Wo = g.out_hw(H, H, k, k)
    dy = torch.randn(N, Ho, Wo, K).bfloat16().to(gpu)
    ext().conv_set_glds_mode(2)
    try:
        r0 = C.conv_dgrad(dy, w, (N, H, H, Cin), g)
        r1 = C.conv_dgrad(dy, w, (N, H, H, Cin), g, w_t=w.permute(1, 2, 3, 0).contiguous())
    finally:
        ext().conv_set_glds_mode(-1)
    assert torch.equal(r0, r1)


@pytest.mark.parametrize("shape", [(8, 14, 14, 256, 256, 3, 1, (1, 1, 1, 1)),
                                   (16, 14, 14, 1024, 256, 1, 1, (0, 0, 0, 0)),
                                   (8, 15, 15, 128, 192, 3, 2, (1, 1, 1, 1))])
def test_conv_m32_kloop(gpu, shape):
    """The 32×32×16-MFMA K loop (TDL_M32, conv_glds_kernel M32: accumulators re-laid to the
    16×16 fragment layout before the shared epilogue) vs the default 16×16×32 loop: forward with
    bias + BN statistics and the transposed-weight dgrad.  The 16×16×32 instruction sums its 32
    products in two 16-deep passes, so the two loops round identically: the outputs are equal."""
    N, H, _, Cin, K, k, s, pad = shape
    g = C.ConvGeom((s, s), pad, (1, 1))
    torch.manual_seed(8)
    x = torch.randn(N, H, H, Cin).bfloat16().to(gpu)
    w = (torch.randn(K, k, k, Cin) * 0.05).bfloat16().to(gpu)
    b = torch.randn(K, device=gpu)
    Ho, Wo = g.out_hw(H, H, k, k)
    dy = torch.randn(N, Ho, Wo, K).bfloat16().to(gpu)
    wt = w.permute(1, 2, 3, 0).contiguous()
    outs = []
    ext().conv_set_glds_mode(2)
    try:
        for m32 in (0, 1):
            ext().conv_set_m32(m32)
            st = torch.zeros(2, K, device=gpu)
            y = C.conv_fwd(x, w, g, bias=b, relu=True, stats=st)
            dx = C.conv_dgrad(dy, w, (N, H, H, Cin), g, w_t=wt)
            outs.append((y, st, dx))
    finally:
        ext().conv_set_m32(-1)
        ext().conv_set_glds_mode(-1)
    (y0, s0, d0), (y1, s1, d1) = outs
    ref = torch.relu(C.ref_conv_fwd(x.cpu(), w.cpu(), g, b.cpu()))
    assert rel_err(y1, ref) < 1e-2
    assert rel_err(d1, C.ref_conv_dgrad(dy.cpu(), w.cpu(), (N, H, H, Cin), g)) < 1e-2
    assert torch.equal(y0, y1) and torch.equal(d0, d1)
    assert rel_err(s1, s0) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(8, 28, 128, 512, 1, 1, (0, 0, 0, 0)),
                                   (8, 14, 256, 256, 3, 1, (1, 1, 1, 1)),
                                   (8, 28, 256, 256, 3, 2, (0, 1, 0, 1)),
                                   (8, 19, 728, 728, 1, 1, (0, 0, 0, 0)),
                                   (3, 9, 64, 200, 3, 1, (1, 1, 1, 1))])
@pytest.mark.parametrize("bias", [False, True])
def test_conv_producer_consumer_fwd(gpu, shape, bias):
    """Wave-specialised producer/consumer forward (conv_pc.hip, TDL_CONV_PC) vs the default
    LDS-DMA forward: same LDS images, fragment order and epilogue — outputs bit-identical,
    fused BN statistics equal up to the atomic order; ragged 728-channel 1×1, strided 3×3,
    partial tiles and column-ragged output channels included."""
    N, H, Cin, K, k, s, pad = shape
    g = C.ConvGeom((s, s), pad, (1, 1))
    torch.manual_seed(9)
    x = torch.randn(N, H, H, Cin).bfloat16().to(gpu)
    w = (torch.randn(K, k, k, Cin) * 0.05).bfloat16().to(gpu)
    b = torch.randn(K, device=gpu) if bias else None
    outs = []
    ext().conv_set_glds_mode(2)
    try:
        for pc in (0, 1, 2):  # conv_glds, 2 producer waves, 4 producer waves
            ext().conv_set_pc(pc)
            st = torch.zeros(2, K, device=gpu)
            y = C.conv_fwd(x, w, g, bias=b, relu=bias, stats=st)
            outs.append((y, st))
    finally:
        ext().conv_set_pc(-1)
        ext().conv_set_glds_mode(-1)
    y0, s0 = outs[0]
    ref = C.ref_conv_fwd(x.cpu(), w.cpu(), g, None if b is None else b.cpu())
    for y1, s1 in outs[1:]:
        assert rel_err(y1, torch.relu(ref) if bias else ref) < 1e-2
        assert torch.equal(y0, y1)
        assert rel_err(s1, s0) < 1e-5


def test_row_packed_stem_gpu(gpu):
    """The row-pack HIP kernel = its CPU oracle (bitwise), and the packed 7×7/s2 stem
    (RowPackedConv2d) = the plain conv on the 8-channel padded input: forward and dW on the GPU."""
    from tensorflowdistributedlearning_amd.models.layers import Conv2d, RowPackedConv2d
    torch.manual_seed(6)
    x = torch.randn(4, 45, 50, 8).bfloat16()
    x[..., 3:] = 0
    for sw, pl, Wo in ((2, 3, 25), (1, 3, 50)):
        ref = C.row_pack(x, 3, 7, sw, pl, Wo, 24)
        got = C.row_pack(x.to(gpu), 3, 7, sw, pl, Wo, 24)
        assert torch.equal(got.cpu(), ref)
    xs = torch.randn(2, 5, 224, 8).bfloat16()  # the ResNet stem's row width (LDS-staged kernel)
    xs[..., 3:] = 0
    assert torch.equal(C.row_pack(xs.to(gpu), 3, 7, 2, 3, 112, 24).cpu(),
                       C.row_pack(xs, 3, 7, 2, 3, 112, 24))
    plain = Conv2d(3, 64, 7, 2, "sym", pad_cin_to=8).to(gpu)
    packed = RowPackedConv2d(3, 64, 7, 2, "sym", pad_cin_to=8).to(gpu)
    packed.weight.data.copy_(plain.weight.data)
    xg = torch.randn(8, 64, 64, 8, device=gpu).bfloat16()
    xg[..., 3:] = 0
    y0, y1 = plain(xg), packed(xg)
    assert rel_err(y1, y0) < 1e-2
    g = torch.randn_like(y0)
    (y0.float() * g.float()).sum().backward()
    (y1.float() * g.float()).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(packed.weight.grad, plain.weight.grad) < 1e-2


def test_maxpool_bwd_bnstat(gpu):
    """Max-pool backward with the producing BN's ReLU mask and its backward sums fused
    (maxpool_bwd_stats): dx = plain gathered dx · [bit] exactly, (Σg, Σg·x) vs fp32."""
    torch.manual_seed(23)
    N, H, W, Cc = 4, 30, 30, 64
    x = (torch.randn(N, H, W, Cc) * 1.2 + 0.2).bfloat16().to(gpu)  # BN input
    coef = B.bn_finalize(B.bn_stats(x), N * H * W, torch.ones(Cc, device=gpu),
                         torch.zeros(Cc, device=gpu), torch.zeros(Cc, device=gpu),
                         torch.ones(Cc, device=gpu), 0.9, 1e-3, True)
    mask = torch.empty(x.numel() // 8, device=gpu, dtype=torch.uint8)
    y = B.bn_apply(x, coef, None, True, mask=mask)
    pad = (1, 1, 1, 1)
    pooled = P.max_pool2d(y, 3, 2, pad)
    dy = torch.randn_like(pooled)
    idx = torch.empty(pooled.shape, device=gpu, dtype=torch.uint8)
    ext().maxpool_fwd(y, torch.empty_like(pooled), idx, 3, 2, 1, 1)
    plain = torch.empty_like(y)
    ext().maxpool_bwd(dy, idx, plain, 3, 2, 1, 1)
    keep = B.unpack_relu_mask(mask, Cc).reshape(y.shape)
    dx = torch.empty_like(y)
    red = torch.zeros(2, Cc, device=gpu)
    assert ext().maxpool_bwd_stats(dy, idx, dx, 3, 2, 1, 1, x, mask, red)
    assert torch.equal(dx, (plain.float() * keep).bfloat16())
    gf, xf = dx.float().reshape(-1, Cc), x.float().reshape(-1, Cc)
    assert rel_err(red, torch.stack([gf.sum(0), (gf * xf).sum(0)])) < 1e-4


def test_bn_bwd_reduce2_matches_two_reduces(gpu):
    """One pass for the two BNs of a downsampling bottleneck (residual BN + shortcut BN, same
    gradient): (Σg, Σg·x̂) of x and raw (Σg, Σg·x2) = two separate reduce passes."""
    torch.manual_seed(29)
    Cc = 256
    x = (torch.randn(8, 14, 14, Cc) + 0.3).bfloat16().to(gpu)
    x2 = (torch.randn(8, 14, 14, Cc) * 0.7 - 0.2).bfloat16().to(gpu)
    dy = torch.randn(8, 14, 14, Cc).bfloat16().to(gpu)
    M = 8 * 14 * 14
    mk = lambda t: B.bn_finalize(B.bn_stats(t), M, torch.ones(Cc, device=gpu),  # noqa: E731
                                 torch.zeros(Cc, device=gpu), torch.zeros(Cc, device=gpu),
                                 torch.ones(Cc, device=gpu), 0.9, 1e-3, True)
    c1, c2 = mk(x), mk(x2)
    red, red2 = B.bn_bwd_reduce2(dy, x, c1, x2)
    torch.testing.assert_close(red, B.bn_bwd_reduce(dy, None, x, c1, 0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(B.bn_red_xhat(red2, c2), B.bn_bwd_reduce(dy, None, x2, c2, 0),
                               rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("C,ld,c0", [(256, 1280, 512), (48, 304, 256), (728, 1456, 0)])
def test_bn_and_upsample_channel_slice_io(gpu, C, ld, c0):
    """The concat-free ASPP / decoder kernels: bn_apply writing into a channel slice of a wider
    NHWC buffer, bn_bwd_reduce / bn_bwd_apply and upsample_bwd reading dy from one, and
    upsample_fwd writing into one, are bitwise the contiguous kernels (other channels untouched)."""
    torch.manual_seed(1)
    N, H, W = 2, 13, 13
    x = torch.randn(N, H, W, C, device=gpu).bfloat16()
    stats = B.bn_stats(x)
    g = torch.rand(C, device=gpu) + 0.5
    b = torch.randn(C, device=gpu) * 0.1
    rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    coef = B.bn_finalize(stats, N * H * W, g, b, rm, rv, 0.9, 1e-3, True)
    y = B.bn_apply(x, coef, None, True)
    buf = torch.full((N, H, W, ld), 7.0, device=gpu, dtype=torch.bfloat16)
    B.bn_apply(x, coef, None, True, out=buf[..., c0:c0 + C])
    torch.cuda.synchronize()
    assert torch.equal(buf[..., c0:c0 + C], y)
    rest = torch.cat([buf[..., :c0], buf[..., c0 + C:]], -1)
    assert torch.all(rest == 7.0)
    gbuf = torch.randn(N, H, W, ld, device=gpu).bfloat16()
    dy = gbuf[..., c0:c0 + C]
    for relu in (0, 2):
        r1 = B.bn_bwd_reduce(dy.contiguous(), None, x, coef, relu)
        r2 = B.bn_bwd_reduce(dy, None, x, coef, relu)
        torch.testing.assert_close(r1, r2, rtol=1e-5, atol=1e-3)
        d1, _ = B.bn_bwd_apply(dy.contiguous(), None, x, coef, r1, g, N * H * W, relu, False)
        d2, _ = B.bn_bwd_apply(dy, None, x, coef, r1, g, N * H * W, relu, False)
        assert torch.equal(d1, d2)
    small = torch.randn(N, 5, 5, C, device=gpu).bfloat16()
    up = U.upsample(small, (H, W))
    buf2 = torch.zeros(N, H, W, ld, device=gpu, dtype=torch.bfloat16)
    U.upsample_into(buf2, c0, small)
    assert torch.equal(buf2[..., c0:c0 + C], up)
    ih, wh = U._tap_tensor(5, H, gpu)
    iw, ww = U._tap_tensor(5, W, gpu)
    dx1 = torch.empty_like(small)
    dx2 = torch.empty_like(small)
    ext().upsample_bwd(dy.contiguous(), dx1, ih, wh, iw, ww)
    ext().upsample_bwd(dy, dx2, ih, wh, iw, ww)
    assert torch.equal(dx1, dx2)


@pytest.mark.parametrize("shape", [(8, 19, 19, 728, 728), (4, 19, 19, 1024, 728),
                                   (4, 10, 10, 728, 1024)])
def test_conv_dgrad_bnstat_ragged_k(gpu, shape):
    """Fused BN-backward statistics on the ragged-K (K % 64 != 0) 1×1 LDS-DMA dgrad — Xception's
    728-channel pointwise convs with a statistics-only token (no ReLU mask): dx bit-identical to
    the plain dgrad, (Σg, Σg·x) vs an fp32 reduction."""
    N, H, W, Cin, K = shape
    g = C.ConvGeom((1, 1), (0, 0, 0, 0), (1, 1))
    torch.manual_seed(23)
    w = (torch.randn(K, 1, 1, Cin) / math.sqrt(Cin)).bfloat16().to(gpu)
    dy = torch.randn(N, H, W, K).bfloat16().to(gpu)
    x = (torch.randn(N, H, W, Cin) * 1.3 + 0.4).bfloat16().to(gpu)
    ext().conv_set_glds_mode(2)
    try:
        ref = C.conv_dgrad(dy, w, x.shape, g)
        dx, red = C.conv_dgrad_bnstat(dy, w, x.shape, g, x)
    finally:
        ext().conv_set_glds_mode(-1)
    assert torch.equal(dx, ref)
    assert red is not None
    gf, xf = dx.float().reshape(-1, Cin), x.float().reshape(-1, Cin)
    want = torch.stack([gf.sum(0), (gf * xf).sum(0)])
    assert rel_err(red, want) < 1e-4


@pytest.mark.parametrize("Cn,stride,H", [(728, 1, 19), (128, 1, 19), (64, 2, 19), (200, 1, 19),
                                        (1536, 1, 2), (728, 1, 4), (256, 1, 7)])
def test_depthwise_fused_bn_stats(gpu, Cn, stride, H):
    """The depthwise kernels' fused BN sums: forward (Σy, Σy²) of the stored output (tile kernel;
    the strided row kernels fall back to a reduce pass inside the op), and the dgrad's
    (Σg, Σg·x_bn) of the stored, x>0-masked dx — vs fp32 reductions; dx bit-identical to the
    unfused dgrad."""
    torch.manual_seed(24)
    from tensorflowdistributedlearning_amd.models.layers import resolve_padding
    pad = resolve_padding("SAME", H, H, 3, 3, (stride, stride), (1, 1))
    g = C.ConvGeom((stride, stride), pad, (1, 1))
    x = torch.randn(4, H, H, Cn, device=gpu).bfloat16()
    w = (torch.randn(3, 3, Cn, device=gpu) * 0.3).bfloat16()
    wp = torch.nn.Parameter(w.float())
    wp._lowp = w
    D.DW_STATS = True
    try:
        y, st = D.depthwise_conv2d(x, wp, None, g, False, want_stats=True)
    finally:
        D.DW_STATS = False
    yf = y.float().reshape(-1, Cn)
    assert rel_err(st, torch.stack([yf.sum(0), (yf * yf).sum(0)])) < 1e-4
    Ho = y.shape[1]
    dy = torch.randn(4, Ho, Ho, Cn, device=gpu).bfloat16()
    bn_x = (torch.randn(4, H, H, Cn, device=gpu) + 0.3).bfloat16()
    dx0 = torch.empty_like(x)
    ext().dwconv_dgrad(dy, w, dx0, stride, stride, pad[0], pad[2], 1, 1, x)
    dx1 = torch.empty_like(x)
    red = torch.zeros(2, Cn, device=gpu)
    fused = ext().dwconv_dgrad(dy, w, dx1, stride, stride, pad[0], pad[2], 1, 1, x, bn_x, red)
    assert torch.equal(dx0, dx1)
    assert fused == (stride == 1 and Cn % 8 == 0)
    if fused:
        gf, xf = dx1.float().reshape(-1, Cn), bn_x.float().reshape(-1, Cn)
        assert rel_err(red, torch.stack([gf.sum(0), (gf * xf).sum(0)])) < 1e-4


def test_bn_bwd_apply_dadd(gpu):
    """bn_bwd_apply(dadd=g2): dx + g2 in the same pass — equals the plain dx plus g2 (bf16
    rounding of the sum once instead of twice)."""
    torch.manual_seed(31)
    M, Cn = 4 * 13 * 13, 1024
    x = torch.randn(4, 13, 13, Cn, device=gpu).bfloat16()
    dy = torch.randn_like(x)
    g2 = torch.randn_like(x)
    gam = torch.rand(Cn, device=gpu) + 0.5
    coef = B.bn_finalize(B.bn_stats(x), M, gam, torch.zeros(Cn, device=gpu),
                         torch.zeros(Cn, device=gpu), torch.ones(Cn, device=gpu), 0.9, 1e-3, True)
    red = B.bn_bwd_reduce(dy, None, x, coef, 2)
    d0, _ = B.bn_bwd_apply(dy, None, x, coef, red, gam, M, 2, False)
    d1, _ = B.bn_bwd_apply(dy, None, x, coef, red, gam, M, 2, False, dadd=g2)
    assert rel_err(d1, d0.float() + g2.float()) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_join_dadd_kernels(gpu, dtype):
    """Residual-gradient join inputs: the depthwise dgrad and the global-average-pool backward add
    an earlier contribution (``dadd``, here in place: out is dadd) in their epilogues — equal to
    the plain result plus that contribution."""
    torch.manual_seed(9)
    N, H, W, Cn = 2, 13, 13, 64
    dy = torch.randn(N, H, W, Cn, device=gpu).to(dtype)
    w = (torch.randn(3, 3, Cn, device=gpu) * 0.3).to(dtype)
    prev = torch.randn(N, H, W, Cn, device=gpu).to(dtype)
    for dil in (1, 2):
        plain = torch.empty_like(prev)
        ext().dwconv_dgrad(dy, w, plain, 1, 1, dil, dil, dil, dil)
        buf = prev.clone()
        ext().dwconv_dgrad(dy, w, buf, 1, 1, dil, dil, dil, dil, dadd=buf)
        tol = 0 if dtype == torch.float32 else 1e-2
        assert rel_err(buf, plain.float() + prev.float()) <= max(tol, 1e-6), dil
    g = torch.randn(N, Cn, device=gpu).to(dtype)
    plain = torch.empty_like(prev)
    ext().avgpool_bwd(g, plain)
    buf = prev.clone()
    ext().avgpool_bwd(g, buf, buf)
    assert rel_err(buf, plain.float() + prev.float()) <= (1e-6 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("hw,c,stride,relu_in", [(75, 256, 1, False), (150, 64, 1, True),
                                                 (38, 728, 1, False), (75, 128, 2, False),
                                                 (38, 256, 2, True), (19, 1024, 2, False)])
def test_depthwise_tiles_at_xception_scale(gpu, hw, c, stride, relu_in):
    """The LDS tile kernels on Xception-sized maps — several tile bands and column tiles per image
    (tiles as tall as 64 KiB of LDS allows), ragged last tiles, 728 = 11·64 + 24 channels —
    forward, input gradient and the tile weight gradient (stride 1 and 2) against fp32 PyTorch."""
    from tensorflowdistributedlearning_amd.models.layers import resolve_padding
    torch.manual_seed(hw + c + stride)
    pad = resolve_padding("SAME" if stride == 1 else (1, 1, 1, 1), hw, hw, 3, 3,
                          (stride, stride), (1, 1))
    g = C.ConvGeom((stride, stride), pad, (1, 1))
    x = torch.randn(2, hw, hw, c).bfloat16()
    w = (torch.randn(3, 3, c) * 0.3).bfloat16()
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = D.ref_dw_fwd(torch.relu(xr) if relu_in else xr, wr, g)
    wp = torch.nn.Parameter(w.float().to(gpu))
    wp._lowp = w.to(gpu)
    xg = x.to(gpu).requires_grad_(True)
    y = D.depthwise_conv2d(xg, wp, None, g, False, relu_in)
    assert rel_err(y, yr) < 2e-2
    dy = torch.randn(yr.shape).bfloat16()
    yr.backward(dy.float())
    y.backward(dy.to(gpu))
    assert rel_err(xg.grad, xr.grad) < 2e-2
    assert rel_err(wp.grad, wr.grad) < 2e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_softmax_eval_head(gpu, dtype):
    """The forward-only classification head (evaluation / prediction): CE sum, top-1 count (first
    maximal index, ties included) and fp32 probabilities vs the fp32 reference."""
    torch.manual_seed(4)
    logits = (torch.randn(37, 1000) * 3).to(dtype)
    logits[5, 10] = logits[5, 20] = logits[5].float().max() + 1  # a tie: argmax is the first
    labels = torch.randint(0, 1000, (37,))
    labels[5] = 10
    labels[:8] = logits[:8].float().argmax(-1)
    ls, cr, p = L.softmax_eval(logits.to(gpu), labels.to(gpu), probs=True)
    lf = logits.float()
    ref_ls = (torch.logsumexp(lf, -1) - lf.gather(1, labels.view(-1, 1)).view(-1)).sum()
    assert abs(float(ls) - float(ref_ls)) < 1e-4 * float(ref_ls)
    assert float(cr) == float((lf.argmax(-1) == labels).sum())
    assert rel_err(p, torch.softmax(lf, -1)) < 1e-5
    _, _, p2 = L.softmax_eval(logits.to(gpu), probs=True)
    assert torch.equal(p2, p)


# (N, H, W, Cin, K, k, dilation): stride-1 dgrads the forward kernels take (K % 64 == 0)
AS_FWD_SHAPES = [
    (4, 14, 14, 64, 64, 3, 1),      # 256x64 8-wave tiles
    (4, 14, 14, 128, 128, 3, 1),
    (4, 14, 14, 256, 256, 3, 1),    # producer/consumer kernel (C_in of the forward = K >= 256)
    (4, 14, 14, 256, 64, 1, 1),
    (4, 14, 14, 64, 256, 1, 1),
    (3, 9, 9, 128, 128, 3, 1),      # ragged last row tile
    (2, 13, 13, 64, 128, 3, 2),     # dilated
]


@pytest.mark.parametrize("shape", AS_FWD_SHAPES)
@pytest.mark.parametrize("epi", ["plain", "mask", "join", "bnstat"])
def test_conv_dgrad_as_forward(gpu, shape, epi):
    """A stride-1 input gradient computed as the forward conv of dy with the flipped filter
    (conv_glds.hip conv_dgrad_as_fwd, models.layers.Conv2d.flip_weight) against the DGRAD kernel
    and the fp32 oracle, for every DGRAD epilogue it carries: plain, ReLU bit mask, residual join
    (dx += …, masked) and the fused BN-backward statistics (Σg, Σg·x)."""
    N, H, W, Cin, K, k, d = shape
    p = d * (k - 1) // 2
    g = C.ConvGeom((1, 1), (p, p, p, p), (d, d))
    torch.manual_seed(41)
    w = (torch.randn(K, k, k, Cin) / math.sqrt(k * k * Cin)).bfloat16().to(gpu)
    wf = torch.empty(Cin, k, k, K, device=gpu, dtype=torch.bfloat16)
    ext().conv_flip_weight(w, wf)
    assert torch.equal(wf, w.flip(1, 2).permute(3, 1, 2, 0))
    dy = torch.randn(N, H, W, K).bfloat16().to(gpu)
    x = (torch.randn(N, H, W, Cin) * 1.3 + 0.4).bfloat16().to(gpu)
    mask = None
    if epi != "plain":
        gam, bet = torch.rand(Cin, device=gpu) + 0.5, torch.randn(Cin, device=gpu) * 0.3
        coef = B.bn_finalize(B.bn_stats(x), N * H * W, gam, bet, torch.zeros(Cin, device=gpu),
                             torch.ones(Cin, device=gpu), 0.9, 1e-3, True)
        mask = torch.empty(x.numel() // 8, device=gpu, dtype=torch.uint8)
        B.bn_apply(x, coef, None, True, mask=mask)
    prev = torch.randn(N, H, W, Cin).bfloat16().to(gpu) if epi == "join" else None
    ext().conv_set_glds_mode(2)
    try:
        if epi == "bnstat":
            ref, red0 = C.conv_dgrad_bnstat(dy, w, x.shape, g, x, mask=mask)
            got, red1 = C.conv_dgrad_bnstat(dy, w, x.shape, g, x, mask=mask, w_flip=wf)
        else:
            ref = C.conv_dgrad(dy, w, x.shape, g, mask=mask,
                               out=prev.clone() if prev is not None else None,
                               accumulate=prev is not None)
            got = C.conv_dgrad(dy, w, x.shape, g, mask=mask, w_flip=wf,
                               out=prev.clone() if prev is not None else None,
                               accumulate=prev is not None)
    finally:
        ext().conv_set_glds_mode(-1)
    torch.cuda.synchronize()
    oracle = C.ref_conv_dgrad(dy.float().cpu(), w.float().cpu(), x.shape, g)
    if prev is not None:
        oracle = oracle + prev.float().cpu()
    if mask is not None:
        oracle = oracle * B.unpack_relu_mask(mask.cpu(), Cin).reshape(oracle.shape)
    assert rel_err(got, oracle) < 1e-2
    assert rel_err(got, ref) < 1e-2
    if epi == "bnstat":
        assert red0 is not None and red1 is not None
        gf, xf = got.float().reshape(-1, Cin), x.float().reshape(-1, Cin)
        want = torch.stack([gf.sum(0), (gf * xf).sum(0)])
        assert rel_err(red1, want) < 1e-4


@pytest.mark.parametrize("shape", [(4, 14, 14, 128, 256, 1, 1, 1, 0),    # 1x1, 256x128 tiles
                                   (4, 14, 14, 64, 128, 3, 3, 1, 1),     # 3x3, <= 128 outputs: 128x128
                                   (3, 15, 15, 256, 512, 3, 3, 2, 1),    # 3x3 / s2, ragged pixels
                                   (2, 9, 11, 48, 144, 1, 1, 2, 0),      # C, K % 16 only
                                   (8, 28, 28, 256, 64, 1, 1, 1, 0)])    # many pixels, split-K
def test_conv_wgrad_fp8(gpu, shape):
    """fp8 weight gradient (e5m2 dy x e4m3 x through transposed 8-bit LDS reads into the f8f6f4
    MFMA, fp32 split-K slabs x the per-tensor scales) vs the fp32 wgrad of the same dequantised
    operands; accumulate adds onto dW."""
    from tensorflowdistributedlearning_amd.ops import fp8 as F8
    N, H, W, Cin, K, R, S, st, p = shape
    g = C.ConvGeom((st, st), (p, p, p, p), (1, 1))
    torch.manual_seed(23)
    Ho, Wo = g.out_hw(H, W, R, S)
    x = torch.randn(N, H, W, Cin).bfloat16()
    dy = torch.randn(N, Ho, Wo, K).bfloat16()
    x8, sx = F8.quantize_e4m3(x.to(gpu))
    dy8, sdy = F8.quantize_e5m2(dy.to(gpu))
    ref = C.ref_conv_wgrad(F8.dequantize_e5m2(dy8, sdy).cpu(), F8.dequantize(x8, sx).cpu(),
                           (K, R, S, Cin), g)
    out = torch.full((K, R, S, Cin), 3.0, device=gpu)
    ext().conv_wgrad_fp8(dy8.view(torch.uint8), x8.view(torch.uint8), out, sdy, sx,
                         *(st, st, p, p, 1, 1), False)
    torch.cuda.synchronize()
    assert ext().conv_last_route(2).startswith("wgrad.glds.fp8")
    assert rel_err(out, ref) < 1e-3
    acc = torch.ones((K, R, S, Cin), device=gpu)
    ext().conv_wgrad_fp8(dy8.view(torch.uint8), x8.view(torch.uint8), acc, sdy, sx,
                         *(st, st, p, p, 1, 1), True)
    torch.cuda.synchronize()
    assert rel_err(acc, ref + 1.0) < 1e-3
    # quantisation error only vs the bf16 wgrad of the unquantised data
    assert rel_err(out, C.ref_conv_wgrad(dy.float(), x.float(), (K, R, S, Cin), g)) < 0.1


# (N, H, W, Cin, K, k, stride, pad (t, b, l, r)): strided dgrads as one forward conv per parity class
AS_FWD_STRIDED = [
    (4, 28, 28, 128, 128, 3, 2, (1, 1, 1, 1)),   # ResNet 3x3 / s2
    (4, 14, 14, 64, 256, 1, 2, (0, 0, 0, 0)),    # 1x1 / s2: three empty classes (zero fill)
    (3, 15, 17, 128, 64, 3, 2, (1, 1, 1, 1)),    # odd sizes, 64-wide dx
    (2, 16, 16, 64, 128, 3, 2, (0, 1, 0, 1)),    # TF SAME asymmetric padding
    (2, 12, 12, 64, 64, 3, 3, (1, 1, 1, 1)),     # stride 3
]


@pytest.mark.parametrize("shape", AS_FWD_STRIDED)
@pytest.mark.parametrize("epi", ["plain", "mask", "join", "bnstat"])
def test_conv_dgrad_as_forward_strided(gpu, shape, epi):
    """A strided input gradient as one stride-1 forward conv of dy per parity class with that
    class's flipped sub-filter (ops/conv.flip_classes, conv_glds.hip dgrad_as_fwd_strided) vs the
    DGRAD kernel and the fp32 oracle, for every DGRAD epilogue: plain, ReLU bit mask, residual
    join, fused BN-backward statistics."""
    N, H, W, Cin, K, k, s, pad = shape
    g = C.ConvGeom((s, s), pad, (1, 1))
    Ho, Wo = g.out_hw(H, W, k, k)
    torch.manual_seed(43)
    w = (torch.randn(K, k, k, Cin) / math.sqrt(k * k * Cin)).bfloat16().to(gpu)
    wf = C.flip_classes(w, g)
    assert wf.numel() == w.numel()
    dy = torch.randn(N, Ho, Wo, K).bfloat16().to(gpu)
    x = (torch.randn(N, H, W, Cin) * 1.3 + 0.4).bfloat16().to(gpu)
    mask = None
    if epi != "plain":
        gam, bet = torch.rand(Cin, device=gpu) + 0.5, torch.randn(Cin, device=gpu) * 0.3
        coef = B.bn_finalize(B.bn_stats(x), N * H * W, gam, bet, torch.zeros(Cin, device=gpu),
                             torch.ones(Cin, device=gpu), 0.9, 1e-3, True)
        mask = torch.empty(x.numel() // 8, device=gpu, dtype=torch.uint8)
        B.bn_apply(x, coef, None, True, mask=mask)
    prev = torch.randn(N, H, W, Cin).bfloat16().to(gpu) if epi == "join" else None
    ext().conv_set_glds_mode(2)
    try:
        if epi == "bnstat":
            ref, red0 = C.conv_dgrad_bnstat(dy, w, x.shape, g, x, mask=mask)
            got, red1 = C.conv_dgrad_bnstat(dy, w, x.shape, g, x, mask=mask, w_flip=wf)
        else:
            ref = C.conv_dgrad(dy, w, x.shape, g, mask=mask,
                               out=prev.clone() if prev is not None else None,
                               accumulate=prev is not None)
            got = C.conv_dgrad(dy, w, x.shape, g, mask=mask, w_flip=wf,
                               out=prev.clone() if prev is not None else None,
                               accumulate=prev is not None)
        route = ext().conv_last_route(1)
    finally:
        ext().conv_set_glds_mode(-1)
    torch.cuda.synchronize()
    assert route.startswith("dgrad.asfwd.strided"), route
    oracle = C.ref_conv_dgrad(dy.float().cpu(), w.float().cpu(), x.shape, g)
    if prev is not None:
        oracle = oracle + prev.float().cpu()
    if mask is not None:
        # the kernels mask every pixel of a parity class that has taps (whether or not a tap
        # lands in range); pixels of classes without taps keep the joined value unmasked
        rows = torch.tensor([len(t) > 0 for t in C._classes(s, k, pad[0])])[torch.arange(H) % s]
        cols = torch.tensor([len(t) > 0 for t in C._classes(s, k, pad[2])])[torch.arange(W) % s]
        touched = (rows[:, None] & cols[None, :]).reshape(1, H, W, 1)
        keep = B.unpack_relu_mask(mask.cpu(), Cin).reshape(oracle.shape)
        oracle = oracle * (keep | ~touched) if prev is not None else oracle * keep
    assert rel_err(got, oracle) < 1e-2
    assert rel_err(got, ref) < 1e-2
    if epi == "bnstat":
        assert red1 is not None
        gf, xf = got.float().reshape(-1, Cin), x.float().reshape(-1, Cin)
        want = torch.stack([gf.sum(0), (gf * xf).sum(0)])
        assert rel_err(red1, want) < 1e-4


@pytest.mark.parametrize("det", [0, 1])
@pytest.mark.parametrize("H", [30, 112])
def test_bn_relu_max_pool_matches_unfused(gpu, det, H):
    """The stem's BN + ReLU folded into the max-pool (ops/pool.bn_relu_max_pool, pool.hip
    bn_maxpool_fwd_kernel) against the unfused BN apply + max-pool: the pooled output bit for bit
    (same bf16 rounding, same argmax ties), the input gradient and dγ, dβ to fp32 rounding — with
    negative γ (channels whose window maximum is the minimum of z) and in deterministic mode (no
    fused sums: the BN reduces itself)."""
    import copy
    from tensorflowdistributedlearning_amd.models.layers import BatchNorm, resolve_padding
    torch.manual_seed(H + det)
    bn_a = BatchNorm(64).to(gpu)
    with torch.no_grad():
        bn_a.gamma.uniform_(-1.0, 2.0)
        bn_a.beta.normal_(0, 0.5)
    bn_b = copy.deepcopy(bn_a)
    z0 = (torch.randn(4, H, H, 64) * 1.5 + 0.3).bfloat16().to(gpu)
    pad = resolve_padding("sym", H, H, 3, 3, (2, 2), (1, 1))
    Ho = (H + pad[0] + pad[1] - 3) // 2 + 1
    dy = torch.randn(4, Ho, Ho, 64).bfloat16().to(gpu)
    ext().det_set(det)
    try:
        st = B.bn_stats(z0)  # one set of batch sums for both (fp32-atomic order otherwise)
        za = z0.clone().requires_grad_(True)
        ref = P.max_pool2d(B.batch_norm_act(za, bn_a, stats=st.clone(), relu=True), 3, 2, pad)
        ref.backward(dy)
        zb = z0.clone().requires_grad_(True)
        assert P.bn_relu_max_pool_ok(zb, bn_b)
        y = P.bn_relu_max_pool(zb, st.clone(), bn_b, 3, 2, pad)
        y.backward(dy)
        torch.cuda.synchronize()
    finally:
        ext().det_set(-1)
    assert torch.equal(y, ref)
    assert rel_err(zb.grad, za.grad) < 1e-2
    # the two-pass fused backward sums every window's fp32 contribution; the unfused gather first
    # stores g per pixel as bf16 (relative rounding 2^-8 per term of Σg·x̂): a few 1e-3 apart
    tol = 1e-3 if det else 5e-3
    assert rel_err(bn_b.gamma.grad, bn_a.gamma.grad) < tol
    assert rel_err(bn_b.beta.grad, bn_a.beta.grad) < tol
    assert torch.allclose(bn_b.running_mean, bn_a.running_mean)
