"""CPU oracle tests: reference-semantics parity of the op layer (TF SAME, subsample folding, TF1
legacy bilinear upsample, Lovász, mIoU formula, BN, optimizers).  NumPy re-implementations of
the reference's TF code paths serve as independent oracles (TF is not installed: parity is pinned
to the reference's documented algorithms)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tensorflowdistributedlearning_amd.ops import conv as C
from tensorflowdistributedlearning_amd.ops import bn as B
from tensorflowdistributedlearning_amd.ops import loss as L
from tensorflowdistributedlearning_amd.ops import upsample as U
from tensorflowdistributedlearning_amd.ops import metrics as Mt
from tensorflowdistributedlearning_amd.ops import optim as O
from tensorflowdistributedlearning_amd.models.layers import resolve_padding


def test_tf_same_padding():
    assert C.same_padding(101, 3, 2) == (1, 1)     # 101 -> 51
    assert C.same_padding(32, 3, 2) == (0, 1)      # even input: asymmetric
    assert C.same_padding(51, 3, 2) == (1, 1)      # pool1 51 -> 26
    assert C.same_padding(13, 3, 1, 2) == (2, 2)   # dilated
    assert C.ConvGeom((2, 2), (1, 1, 1, 1)).out_hw(101, 101, 3, 3) == (51, 51)


def test_subsample_folding_equivalence():
    """3x3 stride-1 SAME conv + 1x1 max-pool stride 2 == stride-2 conv with symmetric padding
    (core/resnet.py:137-140 folded)."""
    torch.manual_seed(0)
    x = torch.randn(2, 26, 26, 8)
    w = torch.randn(4, 3, 3, 8)
    for rate in (1, 2):
        pad = resolve_padding("SAME", 26, 26, 3, 3, (1, 1), (rate, rate))
        full = C.ref_conv_fwd(x, w, C.ConvGeom((1, 1), pad, (rate, rate)))
        sub = full[:, ::2, ::2, :]
        folded = C.ref_conv_fwd(x, w, C.ConvGeom((2, 2), resolve_padding(
            "sym", 26, 26, 3, 3, (2, 2), (rate, rate)), (rate, rate)))
        assert torch.allclose(sub, folded, atol=1e-4)


def test_conv_ref_grads_match_autograd():
    torch.manual_seed(1)
    g = C.ConvGeom((2, 2), (0, 1, 0, 1), (1, 1))
    x = torch.randn(2, 8, 8, 4, requires_grad=True)
    w = torch.randn(6, 3, 3, 4, requires_grad=True)
    y = C.ref_conv_fwd(x, w, g)
    dy = torch.randn_like(y)
    y.backward(dy)
    assert torch.allclose(C.ref_conv_dgrad(dy, w.detach(), x.shape, g), x.grad, atol=1e-4)
    assert torch.allclose(C.ref_conv_wgrad(dy, x.detach(), w.shape, g), w.grad, atol=1e-4)


def _tf1_upsample_numpy(x, out_h, out_w):
    """Literal NumPy replay of core/layers.py _upsample: SYMMETRIC pad 1 → TF1 resize_bilinear
    (align_corners=False, legacy src = dst·in/out) to out+4 → crop [2:-2]."""
    xp = np.pad(x, ((0, 0), (1, 1), (1, 1), (0, 0)), mode="symmetric")
    N, H, W, Cc = xp.shape
    nh, nw = out_h + 4, out_w + 4
    sh, sw = H / nh, W / nw
    out = np.zeros((N, nh, nw, Cc), dtype=np.float64)
    for i in range(nh):
        src = i * sh
        y0 = int(math.floor(src))
        y1 = min(y0 + 1, H - 1)
        fy = src - y0
        for j in range(nw):
            srcx = j * sw
            x0 = int(math.floor(srcx))
            x1 = min(x0 + 1, W - 1)
            fx = srcx - x0
            top = xp[:, y0, x0] * (1 - fx) + xp[:, y0, x1] * fx
            bot = xp[:, y1, x0] * (1 - fx) + xp[:, y1, x1] * fx
            out[:, i, j] = top * (1 - fy) + bot * fy
    return out[:, 2:-2, 2:-2]


@pytest.mark.parametrize("hw,out", [((13, 13), (26, 26)), ((1, 1), (13, 13)),
                                    ((26, 26), (101, 101)), ((5, 7), (9, 12))])
def test_upsample_matches_tf1_legacy(hw, out):
    x = np.random.RandomState(0).randn(2, hw[0], hw[1], 3)
    ref = _tf1_upsample_numpy(x, *out)
    got = U.upsample(torch.tensor(x, dtype=torch.float32), out).numpy()
    assert np.abs(got - ref).max() < 1e-5


def _np_lovasz(logit, label):
    """NumPy replay of core/losses.py lovasz_hinge_flat + lovasz_grad."""
    signs = 2.0 * label - 1.0
    errors = 1.0 - logit * signs
    order = np.argsort(-errors, kind="stable")
    es = errors[order]
    gt = label[order]
    gts = gt.sum()
    inter = gts - np.cumsum(gt)
    union = gts + np.cumsum(1 - gt)
    jac = 1.0 - inter / union
    jac[1:] = jac[1:] - jac[:-1]
    return float(np.dot(np.maximum(es, 0), jac))


def test_lovasz_matches_numpy_and_autograd():
    rs = np.random.RandomState(1)
    logits = rs.randn(3, 200).astype(np.float32)
    labels = (rs.rand(3, 200) > 0.5).astype(np.float32)
    labels[2] = 0
    loss, grad = L.ref_lovasz_hinge(torch.tensor(logits), torch.tensor(labels))
    ref = np.mean([_np_lovasz(logits[i], labels[i]) for i in range(3)])
    assert abs(loss.item() - ref) < 1e-5
    # closed-form gradient == autograd through the sorted errors (stop_grad on lovasz_grad)
    lt = torch.tensor(logits, requires_grad=True)
    tot = 0
    for i in range(3):
        lab = torch.tensor(labels[i])
        sg = 2 * lab - 1
        err = 1 - lt[i] * sg
        es, perm = torch.sort(err, descending=True, stable=True)
        gvec = L.lovasz_grad(lab[perm]).detach()
        tot = tot + torch.dot(torch.relu(es), gvec)
    (tot / 3).backward()
    assert torch.allclose(grad, lt.grad, atol=1e-6)


def test_lovasz_autograd_function():
    torch.manual_seed(2)
    x = torch.randn(2, 10, 10, 1, requires_grad=True)
    y = (torch.rand(2, 10, 10, 1) > 0.5).float()
    loss = L.lovasz_hinge(x, y)
    loss.backward()
    assert x.grad.shape == x.shape and torch.isfinite(x.grad).all()


def test_miou_reference_formula():
    lab = torch.zeros(2, 4, 4, 1)
    pred = torch.zeros(2, 4, 4, 1)
    lab[0, :2] = 1
    pred[0, :3] = 1  # TP 8, FP 4 -> IoU 2/3
    s, a = Mt.ref_seg_scores(lab, pred)
    iou = 8 / 12
    thr = np.array(Mt.IOU_THRESHOLDS)
    assert abs(s[0].item() - np.mean(iou * (iou > thr))) < 1e-6   # D16 formula (parity)
    assert s[1].item() == 1.0                                      # empty mask, empty pred
    sk, _ = Mt.ref_seg_scores(lab, pred, kaggle=True)
    assert abs(sk[0].item() - np.mean(iou > thr)) < 1e-6
    assert abs(a[0].item() - 12 / 16) < 1e-6


def test_streaming_mean():
    sm = Mt.StreamingMean()
    sm.update(torch.tensor([1.0, 2.0]))
    sm.update(torch.tensor([3.0]))
    assert abs(sm.result().item() - 2.0) < 1e-9


def test_softmax_xent_ref():
    torch.manual_seed(3)
    lg = torch.randn(5, 7, requires_grad=True)
    y = torch.randint(0, 7, (5,))
    loss, grad = L.ref_softmax_xent(lg.detach(), y)
    F.cross_entropy(lg, y).backward()
    assert torch.allclose(loss, F.cross_entropy(lg.detach(), y), atol=1e-6)
    assert torch.allclose(grad, lg.grad, atol=1e-6)
    l2 = L.softmax_cross_entropy(lg.detach().requires_grad_(True), y, 0.1)
    assert torch.allclose(l2, F.cross_entropy(lg.detach(), y, label_smoothing=0.1), atol=1e-5)


def test_bn_reference_against_torch():
    torch.manual_seed(4)
    from tensorflowdistributedlearning_amd.models.layers import BatchNorm
    bn = BatchNorm(6, decay=0.9, eps=1e-3)
    x = torch.randn(3, 5, 5, 6, requires_grad=True)
    r = torch.randn(3, 5, 5, 6, requires_grad=True)
    y = bn(x, residual=r, relu=True)
    dy = torch.randn_like(y)
    y.backward(dy)
    x2 = x.detach().permute(0, 3, 1, 2).requires_grad_(True)
    r2 = r.detach().permute(0, 3, 1, 2).requires_grad_(True)
    g2 = torch.ones(6, requires_grad=True)
    b2 = torch.zeros(6, requires_grad=True)
    rm, rv = torch.zeros(6), torch.ones(6)
    y2 = torch.relu(F.batch_norm(x2, rm, rv, g2, b2, True, 0.1, 1e-3) + r2)
    y2.backward(dy.permute(0, 3, 1, 2))
    assert torch.allclose(y, y2.permute(0, 2, 3, 1), atol=1e-5)
    assert torch.allclose(x.grad, x2.grad.permute(0, 2, 3, 1), atol=1e-5)
    assert torch.allclose(r.grad, r2.grad.permute(0, 2, 3, 1), atol=1e-5)
    assert torch.allclose(bn.gamma.grad, g2.grad, atol=1e-4)
    assert torch.allclose(bn.running_mean, rm, atol=1e-6)
    assert torch.allclose(bn.running_var, rv, atol=1e-5)


def test_tf_adam_formula():
    p = torch.tensor([1.0, -2.0] * 32)
    g = torch.tensor([0.5, 0.1] * 32)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    flags = torch.zeros(1, dtype=torch.uint8)
    lr, b1, b2, eps = 1e-3, 0.9, 0.999, 1e-8
    t = 1
    lr_t = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    O.adam_(p, g, m, v, None, flags, lr_t, b1, b2, eps)
    # TF: m=0.1g, v=0.001g², p -= lr_t·m/(√v+ε)
    exp = torch.tensor([1.0, -2.0] * 32) - lr_t * (0.1 * g) / (torch.sqrt(0.001 * g * g) + eps)
    assert torch.allclose(p, exp, atol=1e-7)


def test_exponential_decay():
    assert O.exponential_decay(1e-3, 0) == 1e-3
    assert abs(O.exponential_decay(1e-3, 10000) - 5e-4) < 1e-12
    assert abs(O.exponential_decay(1e-3, 5000) - 1e-3 * 0.5 ** 0.5) < 1e-12


def test_fastdiv_magic_numbers_exact():
    """Host-generated magic divisors used by the LDS-DMA conv kernels (csrc/kernels/kernels.h)."""
    import random
    from tensorflowdistributedlearning_amd import _native
    ext = _native.load()
    rng = random.Random(0)
    divisors = list(range(1, 3000)) + [rng.randrange(1, 1 << 24) for _ in range(500)] + \
        [7, 14, 28, 56, 112, 3136, 12544, 50176, 802816]
    for d in divisors:
        m, s = ext.fastdiv(d)
        assert m < (1 << 32)
        ns = [0, 1, d - 1, d, d + 1, (1 << 31) - 1] + [rng.randrange(0, 1 << 31) for _ in range(50)]
        for n in ns:
            assert (n * m) >> s == n // d, (n, d)


def test_fp8_quantize_and_conv_reference_cpu():
    import math
    from tensorflowdistributedlearning_amd.ops import fp8 as F8
    from tensorflowdistributedlearning_amd.ops import conv as C
    torch.manual_seed(0)
    x = torch.randn(2, 6, 6, 32)
    y8, s = F8.quantize_e4m3(x)
    assert y8.dtype == torch.float8_e4m3fn and abs(float(s) - float(x.abs().max()) / 448) < 1e-6
    assert float(y8.float().abs().max()) == 448.0
    back = F8.dequantize(y8, s)
    assert ((back - x).abs() <= x.abs() * 0.0625 + 1e-3).all()  # within half an e4m3 ulp
    w = torch.randn(8, 3, 3, 32) / math.sqrt(288)
    w8, sw = F8.quantize_e4m3(w)
    g = C.ConvGeom((1, 1), (1, 1, 1, 1), (1, 1))
    y = C.conv_fwd_fp8(y8, s, w8, sw, g)
    ref = C.ref_conv_fwd(F8.dequantize(y8, s), F8.dequantize(w8, sw), g)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2)


def test_relu_bitmask_layout():
    """Bit j of mask byte i is element 8·i + j (the layout bn_apply's relu mode 3 writes)."""
    import numpy as np
    from tensorflowdistributedlearning_amd.ops.bn import unpack_relu_mask
    g = torch.Generator().manual_seed(0)
    m = torch.rand(6, 24, generator=g) > 0.5
    packed = torch.from_numpy(np.packbits(m.numpy().reshape(-1), bitorder="little"))
    assert torch.equal(unpack_relu_mask(packed, 24), m)


def test_depthwise_relu_in_matches_explicit_relu_cpu():
    """depthwise_conv2d(relu_in=True) ≡ depthwise_conv2d(relu(x)) incl. the input gradient mask;
    and Xception's fused pre-activation placement gives the unfused network's output."""
    from tensorflowdistributedlearning_amd.ops import dwconv as D
    torch.manual_seed(3)
    g = C.ConvGeom((1, 1), (1, 1, 1, 1), (1, 1))
    x = torch.randn(2, 9, 9, 16)
    w = torch.nn.Parameter(torch.randn(3, 3, 16) * 0.3)
    xa = x.clone().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    ya = D.depthwise_conv2d(xa, w, None, g, False, relu_in=True)
    yb = D.depthwise_conv2d(torch.relu(xb), w, None, g, False)
    torch.testing.assert_close(ya, yb)
    dy = torch.randn_like(ya)
    ya.backward(dy)
    yb.backward(dy)
    torch.testing.assert_close(xa.grad, xb.grad)

    from tensorflowdistributedlearning_amd.models.xception import XceptionModule
    m = XceptionModule(16, [16, 16, 16], "sum", 1, 1, [1, 1, 1], False,
                       dict(bn_decay=0.9, bn_eps=1e-3)).eval()
    xi = torch.randn(2, 9, 9, 16)
    with torch.no_grad():
        r = xi
        for conv in m.convs:  # the unfused pre-activation order of core/xception.py:90-110
            r = conv.depthwise(torch.relu(r))
            r = conv.dw_bn(r, relu=False)
            pw = conv.pointwise
            r = pw.bn(pw.conv(r), relu=False)
        ref = r + xi
        torch.testing.assert_close(m(xi), ref, rtol=1e-4, atol=1e-4)


def test_conv_dgrad_bnstat_cpu_oracle():
    """CPU oracle of the fused BN-backward statistics: (Σg, Σg·x) of the stored dx, and
    bn_bwd_apply(red_raw=True) — Σg·x̂ = invstd·(Σg·x − mean·Σg) — equals the reduce path."""
    torch.manual_seed(3)
    g = C.ConvGeom((1, 1), (1, 1, 1, 1), (1, 1))
    x = torch.randn(2, 9, 9, 16) * 1.2 + 0.5
    w = torch.randn(24, 3, 3, 16) * 0.1
    dy = torch.randn(2, 9, 9, 24)
    dx, red = C.conv_dgrad_bnstat(dy, w, x.shape, g, x)
    assert torch.allclose(dx, C.conv_dgrad(dy, w, x.shape, g))
    gf, xf = dx.reshape(-1, 16), x.reshape(-1, 16)
    assert torch.allclose(red, torch.stack([gf.sum(0), (gf * xf).sum(0)]), atol=1e-4)
    st = B.bn_stats(x)
    coef = B.bn_finalize(st, 162, torch.ones(16), torch.zeros(16), torch.zeros(16),
                         torch.ones(16), 0.9, 1e-3, True)
    want = B.bn_bwd_reduce(dx, None, x, coef, 0)
    assert torch.allclose(B.bn_red_xhat(red, coef), want, rtol=1e-4, atol=1e-4)
    gam = torch.rand(16) + 0.5
    d0, _ = B.bn_bwd_apply(dx, None, x, coef, want, gam, 162, 0, False)
    d1, _ = B.bn_bwd_apply(dx, None, x, coef, red, gam, 162, 0, False, red_raw=True)
    assert torch.allclose(d0, d1, rtol=1e-4, atol=1e-5)
    # strided dgrads fuse (parity classes) unless they accumulate into a join
    g2 = C.ConvGeom((2, 2), (1, 1, 1, 1))
    dx2, r2 = C.conv_dgrad_bnstat(dy[:, ::2, ::2].contiguous(), w, x.shape, g2, x)
    assert r2 is not None and torch.allclose(r2[0], dx2.reshape(-1, 16).sum(0), atol=1e-4)
    _, r3 = C.conv_dgrad_bnstat(dy[:, ::2, ::2].contiguous(), w, x.shape, g2, x, out=dx2.clone(),
                                accumulate=True)
    assert r3 is None


def test_row_packed_stem_matches_conv():
    """RowPackedConv2d (7×7/s2 stem as a 7×1 conv over the row-packed image) = the plain conv on
    the 8-channel padded input: forward and weight gradient (CPU oracle path)."""
    from tensorflowdistributedlearning_amd.models.layers import Conv2d, RowPackedConv2d
    torch.manual_seed(4)
    plain = Conv2d(3, 16, 7, 2, "sym", pad_cin_to=8)
    packed = RowPackedConv2d(3, 16, 7, 2, "sym", pad_cin_to=8)
    packed.weight.data.copy_(plain.weight.data)
    for H, W in ((32, 32), (29, 35)):
        x = torch.randn(2, H, W, 8)
        x[..., 3:] = 0
        y0 = plain(x)
        y1 = packed(x)
        assert y1.shape == y0.shape
        assert torch.allclose(y0, y1, atol=1e-4, rtol=1e-4)
        g = torch.randn_like(y0)
        plain.weight.grad = packed.weight.grad = None
        (y0 * g).sum().backward()
        (y1 * g).sum().backward()
        assert torch.allclose(plain.weight.grad, packed.weight.grad, atol=1e-3, rtol=1e-4)
    t = C.row_pack(x, 3, 7, 2, 3, 18, 24)
    assert t.shape == (2, 29, 18, 24) and float(t[..., 21:].abs().sum()) == 0.0


def test_row_pack_input_gradient():
    """The packed stem's input gradient (the row-pack's transposed gather) = the plain conv's."""
    from tensorflowdistributedlearning_amd.models.layers import Conv2d, RowPackedConv2d
    torch.manual_seed(8)
    plain = Conv2d(3, 8, 7, 2, "sym", pad_cin_to=8)
    packed = RowPackedConv2d(3, 8, 7, 2, "sym", pad_cin_to=8)
    packed.weight.data.copy_(plain.weight.data)
    x = torch.randn(2, 21, 23, 8)
    x[..., 3:] = 0
    x0, x1 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    g = torch.randn(2, 11, 12, 8)
    (plain(x0) * g).sum().backward()
    (packed(x1) * g).sum().backward()
    assert torch.allclose(x0.grad[..., :3], x1.grad[..., :3], atol=1e-4, rtol=1e-4)
