"""BN + ReLU folded into the consuming depthwise conv (ops/dwfold.py, DwArgs::aff): an Xception
module's units 2 and 3 against the unfolded step, and the three depthwise kernels with a folded
input against the materialised-input kernels."""
import copy

import pytest
import torch

from tensorflowdistributedlearning_amd.ops import dwfold
from tensorflowdistributedlearning_amd.models.xception import XceptionModule

BN_KW = dict(bn_decay=0.9, bn_eps=1e-3)


def _module(c=16, device="cpu", seed=0):
    torch.manual_seed(seed)
    m = XceptionModule(c, [c, c, c], "sum", 1, 1, [1, 1, 1], False, BN_KW).to(device)
    with torch.no_grad():
        for conv in m.convs:
            conv.pointwise.bn.gamma.uniform_(0.5, 1.5)
            conv.pointwise.bn.beta.normal_(0, 0.5)
    m.train()
    return m, copy.deepcopy(m)


def _step(m, x, g, fold, monkeypatch):
    monkeypatch.setattr(dwfold, "ENABLED", fold)
    xx = x.detach().clone().requires_grad_(True)
    y = m(xx)
    (y.float() * g).sum().backward()
    return y, xx.grad


def test_deferred_bn_plumbing_cpu(monkeypatch):
    """CPU: the deferred BN is applied by its consumer (materialised: the fold is GPU-only) —
    the module's outputs, gradients and moving statistics are the unfolded ones exactly."""
    a, b = _module()
    x = torch.randn(2, 7, 7, 16)
    g = torch.randn(2, 7, 7, 16)
    ya, gxa = _step(a, x, g, True, monkeypatch)
    yb, gxb = _step(b, x, g, False, monkeypatch)
    torch.testing.assert_close(ya, yb, rtol=0, atol=0)
    torch.testing.assert_close(gxa, gxb, rtol=0, atol=0)
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        torch.testing.assert_close(pa.grad, pb.grad, rtol=0, atol=0, msg=n)
    for (n, ba), (_, bb) in zip(a.named_buffers(), b.named_buffers()):
        torch.testing.assert_close(ba, bb, rtol=0, atol=0, msg=n)


def test_deferred_bn_materializes_for_other_consumers():
    torch.manual_seed(1)
    m, _ = _module()
    z = torch.randn(2, 5, 5, 16)
    d = dwfold.DeferredBNAct(z, None, m.convs[0].pointwise.bn)
    u = d.materialize()
    assert u.shape == z.shape and float(u.min()) >= 0.0
    assert d.shape == z.shape


@pytest.mark.gpu
def test_dwfold_module_matches_unfolded_gpu(monkeypatch, gpu):
    from tensorflowdistributedlearning_amd.models.params import FlatParams
    a, b = _module(c=728, device=gpu)
    for m in (a, b):
        m._flat = FlatParams(m, gpu, lowp_dtype=torch.bfloat16)
    monkeypatch.setattr(dwfold, "ENABLED", True)
    assert dwfold.foldable(torch.empty(8, 19, 19, 728, device=gpu, dtype=torch.bfloat16),
                           a.convs[1].depthwise)
    x = (torch.randn(8, 19, 19, 728, device=gpu) * 2 + 0.3).bfloat16()
    g = torch.randn(8, 19, 19, 728, device=gpu)
    ya, gxa = _step(a, x, g, True, monkeypatch)
    yb, gxb = _step(b, x, g, False, monkeypatch)
    torch.cuda.synchronize()

    def cos(p, q):
        p, q = p.float().flatten(), q.float().flatten()
        return float(p @ q / (p.norm() * q.norm() + 1e-30))
    # the kernels are exact (test below), but the BN statistics are fp32 atomic sums in run order
    # (two unfolded runs differ the same way), and bf16 rounding flips propagate from there
    assert cos(ya, yb) > 0.999
    assert (ya.float() - yb.float()).abs().mean() < 1e-2 * yb.float().abs().mean()
    assert cos(gxa, gxb) > 0.999
    pa_all = dict(a.named_parameters())
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        if n.endswith("dw_bn.beta"):
            # analytically zero (the depthwise BN is folded into a pointwise conv that feeds a
            # training BN, ops/bnfold.py): rounding noise in both runs
            ref = float(pa_all[n[:-4] + "gamma"].grad.abs().max())
            assert pa.grad.abs().max() < 1e-2 * ref and pb.grad.abs().max() < 1e-2 * ref, n
            continue
        assert cos(pa.grad, pb.grad) > 0.999, n
    for (n, ba), (_, bb) in zip(a.named_buffers(), b.named_buffers()):
        # batch statistics of bf16 activations downstream of the rounding flips above; the
        # pointwise BNs' moving means are ~1e-4 (zero-mean inputs): absolute tolerance
        torch.testing.assert_close(ba, bb, rtol=1e-2, atol=1e-3, msg=n)


@pytest.mark.gpu
def test_depthwise_kernels_with_folded_input(gpu):
    """dwconv_fwd / dgrad / wgrad with ``aff`` = the materialised u = relu(a·z + b) path."""
    from tensorflowdistributedlearning_amd.ops.common import ext
    torch.manual_seed(5)
    N, H, W, C = 4, 19, 19, 728
    z = (torch.randn(N, H, W, C, device=gpu) * 1.5).bfloat16()
    coef = torch.zeros(4, C, device=gpu)
    coef[0].uniform_(0.3, 2.0)
    coef[1].normal_(0, 0.5)
    from tensorflowdistributedlearning_amd.ops.bn import bn_apply
    u = bn_apply(z, coef, None, True, None, None)  # the BN apply pass's u = relu(a·z + b)
    w = (torch.randn(3, 3, C, device=gpu) * 0.3).bfloat16()
    # forward (+ fused output statistics)
    y0, y1 = torch.empty_like(z), torch.empty_like(z)
    s0, s1 = torch.zeros(2, C, device=gpu), torch.zeros(2, C, device=gpu)
    ext().dwconv_fwd(u, w, None, y0, 1, 1, 1, 1, 1, 1, False, False, s0)
    ext().dwconv_fwd(z, w, None, y1, 1, 1, 1, 1, 1, 1, False, False, s1, aff=coef)
    torch.testing.assert_close(y1, y0, rtol=0, atol=0)
    torch.testing.assert_close(s1, s0, rtol=1e-5, atol=0)  # (fp32 atomics: summation order)
    # input gradient: masked by u > 0 (materialised: mask_x = u) vs a·z + b > 0, and the
    # BN-backward sums against bn_x = z
    dy = torch.randn(N, H, W, C, device=gpu).bfloat16()
    d0, d1 = torch.empty_like(z), torch.empty_like(z)
    r0, r1 = torch.zeros(2, C, device=gpu), torch.zeros(2, C, device=gpu)
    ext().dwconv_dgrad(dy, w, d0, 1, 1, 1, 1, 1, 1, u, z, r0)
    ext().dwconv_dgrad(dy, w, d1, 1, 1, 1, 1, 1, 1, None, z, r1, aff=coef)
    torch.testing.assert_close(d1, d0, rtol=0, atol=0)
    torch.testing.assert_close(r1, r0, rtol=1e-5, atol=1e-3)
    # weight gradient on u (relu_in on the materialised u is a no-op) vs the transformed z
    g0 = torch.zeros(3, 3, C, device=gpu)
    g1 = torch.zeros(3, 3, C, device=gpu)
    ext().dwconv_wgrad(dy, u, g0, None, 1, 1, 1, 1, 1, 1, False, False)
    ext().dwconv_wgrad(dy, z, g1, None, 1, 1, 1, 1, 1, 1, False, False, aff=coef)
    torch.testing.assert_close(g1, g0, rtol=0, atol=0)
    # a geometry the kernels cannot take is refused
    assert not ext().dwconv_aff_ok(z, w, 2, 2, 1, 1, 1, 1)
    with pytest.raises(RuntimeError):
        ext().dwconv_fwd(z, w, None, torch.empty(N, 10, 10, C, device=gpu, dtype=torch.bfloat16),
                         2, 2, 1, 1, 1, 1, False, False, None, aff=coef)
