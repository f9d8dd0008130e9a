"""BN + ReLU folded into the consuming dense conv (ops/bnconv.py, ConvArgs::aff): the CPU plumbing
of the autograd function against the unfolded layers, the three conv kernels with a folded input
against the materialised-input kernels (GPU), and a ResNet-50 step folded vs unfolded (GPU)."""
import copy
import math

import pytest
import torch

from tensorflowdistributedlearning_amd.ops import bnconv, conv as C, bn as B
from tensorflowdistributedlearning_amd.models.layers import ConvBN
from tensorflowdistributedlearning_amd.models.resnet import Bottleneck

BN_KW = dict(bn_decay=0.9, bn_eps=1e-3)


def _pair(cin=16, width=24, stride=1, k=3, seed=0):
    """conv1 (1×1) + BN + ReLU feeding conv2 (k×k, stride) + BN, twice (identical copies)."""
    torch.manual_seed(seed)
    m = torch.nn.ModuleDict(dict(
        a=ConvBN(cin, width, 1, 1, 0, relu=True, init="kaiming_fan_out", **BN_KW),
        b=ConvBN(width, width, k, stride, "sym", relu=True, init="kaiming_fan_out", **BN_KW)))
    with torch.no_grad():
        m["a"].bn.gamma.uniform_(0.5, 1.5)
        m["a"].bn.beta.normal_(0, 0.5)
    m.train()
    return m, copy.deepcopy(m)


@pytest.mark.parametrize("stride,k", [(1, 3), (2, 3), (1, 1)])
def test_bn_act_conv_plumbing_cpu(stride, k):
    """The folded autograd function (forced onto the CPU oracle) = conv(relu(BN(z))) of the
    unfolded layers: output, every gradient, the moving statistics."""
    a, b = _pair(stride=stride, k=k)
    x = torch.randn(2, 9, 9, 16)
    Ho = (9 + 2 * ((k - 1) // 2) - k) // stride + 1
    g = torch.randn(2, Ho, Ho, 24)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    # folded: conv1 defers its BN, conv2's layer consumes it through _BNActConvFn
    z, st = a["a"].conv(xa, want_stats=True)
    ya, st2 = bnconv.bn_act_conv(bnconv.DeferredBNAct(z, st, a["a"].bn), a["b"].conv,
                                 want_stats=True, force=True)
    ya = a["b"].bn(ya, stats=st2, relu=True)
    yb = b["b"](b["a"](xb))
    (ya.float() * g).sum().backward()
    (yb.float() * g).sum().backward()
    torch.testing.assert_close(ya, yb, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(xa.grad, xb.grad, rtol=1e-4, atol=1e-5)
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-4, atol=1e-5, msg=n)
    for (n, ba), (_, bb) in zip(a.named_buffers(), b.named_buffers()):
        torch.testing.assert_close(ba, bb, rtol=1e-5, atol=1e-6, msg=n)


def test_bottleneck_defers_and_materializes_on_cpu(monkeypatch):
    """On the CPU the bottleneck's deferred BNs are materialised by their consumers: outputs and
    gradients are the unfolded ones exactly."""
    torch.manual_seed(3)
    m = Bottleneck(32, 8, 2, BN_KW)
    m.train()
    m2 = copy.deepcopy(m)
    x = torch.randn(2, 10, 10, 32)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    monkeypatch.setattr(bnconv, "ENABLED", True)
    ya = m(xa)
    monkeypatch.setattr(bnconv, "ENABLED", False)
    yb = m2(xb)
    ya.sum().backward()
    yb.sum().backward()
    torch.testing.assert_close(ya, yb, rtol=0, atol=0)
    torch.testing.assert_close(xa.grad, xb.grad, rtol=0, atol=0)


def test_deferred_bn_act_is_applied_for_non_conv_consumers():
    m, _ = _pair()
    z = torch.randn(2, 5, 5, 24)
    d = bnconv.DeferredBNAct(z, None, m["a"].bn)
    u = d.materialize()
    assert u.shape == z.shape and float(u.min()) >= 0.0
    assert not bnconv.foldable(z, m["b"].conv)  # CPU: never folded


# ---------------------------------------------------------------------------------------------
# GPU: kernels with a folded input against the materialised-input kernels
# ---------------------------------------------------------------------------------------------

def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-6))


# (N, H, W, C, K, k, stride, glds mode): mode 2 forces the LDS-DMA / producer-consumer kernels
# onto small problems; mode 1 is the default routing (the register-staged kernels here)
AFF_SHAPES = [
    (4, 14, 14, 64, 64, 3, 1, 1),
    (4, 14, 14, 64, 64, 3, 1, 2),
    (4, 14, 14, 128, 128, 3, 1, 2),
    (4, 15, 15, 128, 128, 3, 2, 2),
    (4, 14, 14, 256, 256, 3, 1, 2),
    (4, 14, 14, 64, 256, 1, 1, 2),
    (4, 14, 14, 128, 512, 1, 1, 1),
    (3, 9, 9, 64, 128, 1, 1, 2),     # M = 243: one ragged row tile
    (4, 14, 14, 512, 128, 3, 1, 2),
]


def _aff_problem(gpu, shape, seed=31):
    N, H, W, Cin, K, k, st, mode = shape
    p = (k - 1) // 2
    g = C.ConvGeom((st, st), (p, p, p, p), (1, 1))
    torch.manual_seed(seed)
    z = (torch.randn(N, H, W, Cin) * 1.3 + 0.2).bfloat16().to(gpu)
    coef = torch.zeros(4, Cin, device=gpu)
    coef[0].uniform_(0.3, 2.0)
    coef[1].normal_(0, 0.6)
    w = (torch.randn(K, k, k, Cin) / math.sqrt(k * k * Cin)).bfloat16().to(gpu)
    return g, z, coef, w, mode


def _args(g):
    return (g.stride[0], g.stride[1], g.padding[0], g.padding[2], g.dilation[0], g.dilation[1])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", AFF_SHAPES)
def test_conv_fwd_with_folded_bn(gpu, shape):
    """conv_fwd(z, aff) = conv_fwd(u) with u = the BN apply pass's relu(a·z + b): outputs
    bit-identical (same operand bits, same K order), statistics up to atomic summation order;
    against the fp32 oracle on u."""
    from tensorflowdistributedlearning_amd.ops.common import ext
    g, z, coef, w, mode = _aff_problem(gpu, shape)
    u = B.bn_apply(z, coef, None, True)
    N, H, W, Cin = z.shape
    Ho, Wo = g.out_hw(H, W, w.shape[1], w.shape[2])
    y0 = torch.empty(N, Ho, Wo, w.shape[0], device=gpu, dtype=torch.bfloat16)
    y1 = torch.empty_like(y0)
    s0 = torch.zeros(2, w.shape[0], device=gpu)
    s1 = torch.zeros_like(s0)
    ext().conv_set_glds_mode(mode)
    try:
        ext().conv_fwd(u, w, y0, None, s0, *_args(g), False)
        ext().conv_fwd(z, w, y1, None, s1, *_args(g), False, None, coef)
    finally:
        ext().conv_set_glds_mode(-1)
    torch.cuda.synchronize()
    ref = C.ref_conv_fwd(u.float().cpu(), w.float().cpu(), g)
    assert _rel(y1, ref) < 1e-2
    assert _rel(y1, y0) < 1e-2
    assert (y1 != y0).float().mean().item() < 1e-3, "folded forward differs from materialised"
    assert _rel(s1, s0) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("shape", AFF_SHAPES)
def test_conv_dgrad_with_folded_bn_mask(gpu, shape):
    """conv_dgrad(aff) masks by a·z + b > 0 in the fused-statistics epilogue: dx bit-identical to
    the bit-mask dgrad of the materialised BN, (Σg, Σg·z) equal up to atomic order; when the
    kernel cannot fuse (returns False) dx is the plain unmasked dgrad."""
    from tensorflowdistributedlearning_amd.ops.common import ext
    g, z, coef, w, mode = _aff_problem(gpu, shape)
    N, H, W, Cin = z.shape
    Ho, Wo = g.out_hw(H, W, w.shape[1], w.shape[2])
    torch.manual_seed(7)
    dy = torch.randn(N, Ho, Wo, w.shape[0]).bfloat16().to(gpu)
    mask = torch.empty(z.numel() // 8, device=gpu, dtype=torch.uint8)
    B.bn_apply(z, coef, None, True, mask=mask)
    ext().conv_set_glds_mode(mode)
    try:
        ref, red0 = C.conv_dgrad_bnstat(dy, w, z.shape, g, z, mask=mask)
        plain = C.conv_dgrad(dy, w, z.shape, g)
        dx = torch.empty_like(z)
        red1 = torch.zeros(2, Cin, device=gpu)
        fused = ext().conv_dgrad(dy, w, dx, *_args(g), False, None, None, z, red1, coef)
    finally:
        ext().conv_set_glds_mode(-1)
    torch.cuda.synchronize()
    if not fused:
        assert torch.equal(dx, plain)
        return
    assert red0 is not None
    assert torch.equal(dx, ref)
    assert _rel(red1, red0) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("shape", AFF_SHAPES)
def test_conv_wgrad_with_folded_bn(gpu, shape):
    """conv_wgrad(z, aff) = conv_wgrad(u): fp32 dW up to split-K summation order."""
    from tensorflowdistributedlearning_amd.ops.common import ext
    g, z, coef, w, mode = _aff_problem(gpu, shape)
    u = B.bn_apply(z, coef, None, True)
    N, H, W, Cin = z.shape
    Ho, Wo = g.out_hw(H, W, w.shape[1], w.shape[2])
    torch.manual_seed(9)
    dy = torch.randn(N, Ho, Wo, w.shape[0]).bfloat16().to(gpu)
    ref = C.conv_wgrad(dy, u, tuple(w.shape), g)
    out = torch.full(tuple(w.shape), 7.0, device=gpu)
    ext().conv_wgrad(dy, z, out, None, *_args(g), False, coef)
    acc = torch.ones(tuple(w.shape), device=gpu)
    ext().conv_wgrad(dy, z, acc, None, *_args(g), True, coef)
    torch.cuda.synchronize()
    assert _rel(out, ref) < 1e-4
    assert _rel(acc - 1.0, ref) < 1e-4
    oracle = C.ref_conv_wgrad(dy.float().cpu(), u.float().cpu(), tuple(w.shape), g)
    assert _rel(out, oracle) < 1e-3


@pytest.mark.gpu
def test_resnet50_step_folded_matches_unfolded(gpu, monkeypatch):
    """Two ResNet-50 training steps with the bottleneck BNs folded (32 folds per forward) against
    the unfolded network from the same state: losses, logits and weights agree to the
    run-to-run level of the fp32 statistics atomics."""
    from tensorflowdistributedlearning_amd import models
    from tensorflowdistributedlearning_amd.engine.trainer import Trainer
    from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy
    from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch
    from tensorflowdistributedlearning_amd.ops.common import ext
    torch.manual_seed(17)
    init = models.resnet50(num_classes=10).state_dict()
    x, y = imagenet_batch(8, 64, num_classes=10, device=gpu)
    calls = []
    orig = bnconv._BNActConvFn.forward

    def counting(ctx, *a):
        calls.append(1)
        return orig(ctx, *a)

    res = {}
    for fold in (True, False):
        monkeypatch.setattr(bnconv, "ENABLED", fold)
        monkeypatch.setattr(bnconv._BNActConvFn, "forward", staticmethod(counting))
        calls.clear()
        m = models.resnet50(num_classes=10)
        m.load_state_dict(init)
        tr = Trainer(m, softmax_cross_entropy, gpu, "sgd", dict(lr=0.01, momentum=0.9))
        # deterministic mode: fixed-order BN statistics, so the first forward (before any update)
        # must agree bit for bit; the fused dgrad sums then fall back to reduce passes
        ext().det_set(1)
        try:
            losses = [float(tr.train_step(x, y)[0]) for _ in range(2)]
            torch.cuda.synchronize()
        finally:
            ext().det_set(-1)
        res[fold] = (losses, tr.flat.master.clone(), len(calls))
    assert res[True][2] == 2 * 32 and res[False][2] == 0
    la, lb = res[True][0], res[False][0]
    assert la[0] == lb[0], (la, lb)
    assert abs(la[1] - lb[1]) <= 1e-3 * abs(lb[1]) + 1e-4, (la, lb)
    ma, mb = res[True][1], res[False][1]
    cos = float(ma @ mb / (ma.norm() * mb.norm()))
    assert cos > 0.99999, cos
