"""Training BN folded into its 1×1 consumer conv (ops/bnfold.py) — Xception's depthwise BN →
pointwise conv: forward, every gradient and the moving statistics against the unfolded
BN-apply + conv path (CPU fp32 oracle; GPU bf16 kernels)."""
import copy

import pytest
import torch

from tensorflowdistributedlearning_amd.ops import bnfold
from tensorflowdistributedlearning_amd.models.xception import SeparableConvBN


def _pair(cin=16, cout=24, relu_out=True, device="cpu", seed=0):
    torch.manual_seed(seed)
    m = SeparableConvBN(cin, cout, 1, 1, False, dict(bn_decay=0.9, bn_eps=1e-3),
                        relu_out=relu_out).to(device)
    with torch.no_grad():
        m.dw_bn.gamma.uniform_(0.5, 1.5)
        m.dw_bn.beta.normal_(0, 0.5)
    m.train()
    return m, copy.deepcopy(m)


def _run(m, x, g, fold, monkeypatch, residual=None):
    monkeypatch.setattr(bnfold, "ENABLED", fold)
    xx = x.detach().clone().requires_grad_(True)
    y = m(xx, relu_in=True, residual=residual)
    (y.float() * g).sum().backward()
    return y, xx.grad


@pytest.mark.parametrize("relu_out,res", [(True, False), (False, True)])
def test_fold_matches_unfolded_cpu(monkeypatch, relu_out, res):
    a, b = _pair(relu_out=relu_out)
    x = torch.randn(2, 9, 9, 16) * 2 + 0.3
    r = torch.randn(2, 9, 9, 24) if res else None
    g = torch.randn(2, 9, 9, 24)
    ya, gxa = _run(a, x, g, True, monkeypatch, r)
    yb, gxb = _run(b, x, g, False, monkeypatch, r)
    torch.testing.assert_close(ya, yb, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(gxa, gxb, rtol=1e-4, atol=1e-5)
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        # (the pointwise weight gradient drops b ⊗ Σdy, zero up to fp32 rounding)
        scale = float(pb.grad.abs().max())
        torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-4, atol=1e-5 * max(scale, 1.0),
                                   msg=n)
    for (n, ba), (_, bb) in zip(a.named_buffers(), b.named_buffers()):
        torch.testing.assert_close(ba, bb, rtol=1e-5, atol=1e-6, msg=n)


def test_fold_validates_its_operands():
    a, _ = _pair()
    with pytest.raises(ValueError):
        bnfold.bn_conv1x1(torch.randn(1, 3, 3, 16), None, a.dw_bn.eval(), a.pointwise.conv)


@pytest.mark.gpu
def test_fold_matches_unfolded_gpu(monkeypatch, gpu):
    """bf16 kernels: the folded step against the unfolded one (u rounded to bf16 there, never
    materialised here) — agreement to bf16 rounding, gradients by cosine."""
    from tensorflowdistributedlearning_amd.models.params import FlatParams
    dev = torch.device("cuda", 0)
    a, b = _pair(cin=728, cout=728, device=dev)
    for m in (a, b):
        m._flat = FlatParams(m, dev, lowp_dtype=torch.bfloat16)
    x = (torch.randn(8, 19, 19, 728, device=dev) * 2 + 0.3).bfloat16()
    g = torch.randn(8, 19, 19, 728, device=dev)
    ya, gxa = _run(a, x, g, True, monkeypatch)
    yb, gxb = _run(b, x, g, False, monkeypatch)
    torch.cuda.synchronize()

    def cos(p, q):
        p, q = p.float().flatten(), q.float().flatten()
        return float(p @ q / (p.norm() * q.norm() + 1e-30))
    assert cos(ya, yb) > 0.9999
    assert cos(gxa, gxb) > 0.999
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        if n == "dw_bn.beta":
            # analytically zero: the pointwise conv's output feeds a training BN, whose input
            # gradient sums to zero per channel, so Σ_p du = Wᵀ·Σ_p dy = 0 — both paths hold
            # rounding noise only
            ref = pa.grad.new_tensor(float(a.dw_bn.gamma.grad.abs().max()))
            assert pa.grad.abs().max() < 1e-2 * ref and pb.grad.abs().max() < 1e-2 * ref
            continue
        assert cos(pa.grad, pb.grad) > 0.999, n
    for (n, ba), (_, bb) in zip(a.named_buffers(), b.named_buffers()):
        # the pointwise BN's moving mean sees W·u with u rounded to bf16 (unfolded) vs W'·z + W·b
        rel = float((ba - bb).abs().max() / bb.abs().max().clamp_min(1e-6))
        assert rel < 1e-2, (n, rel)


@pytest.mark.gpu
def test_fold_weight_kernels_match_torch(gpu):
    """csrc/kernels/bnfold.hip: W·diag(a) (bf16 and fp32), bias W·b (+ bias_in), and the in-place
    column scale of the fp32 weight gradient, against PyTorch."""
    from tensorflowdistributedlearning_amd.ops.common import ext
    torch.manual_seed(3)
    K, C, Cp = 300, 728, 736
    coef = torch.randn(4, Cp, device=gpu)
    bi = torch.randn(K, device=gpu)
    for dt in (torch.bfloat16, torch.float32):
        w = torch.randn(K, 1, 1, C, device=gpu).to(dt)
        wf, b = torch.empty_like(w), torch.empty(K, device=gpu)
        ext().bn_fold_weight(w, coef, wf, bi, b)
        w2 = w.float().view(K, C)
        torch.testing.assert_close(wf.float().view(K, C), (w2 * coef[0, :C]).to(dt).float(),
                                   rtol=0, atol=0)
        torch.testing.assert_close(b, w2 @ coef[1, :C] + bi, rtol=1e-5, atol=1e-4)
    dw = torch.randn(K, 1, 1, C, device=gpu)
    ref = dw.view(K, C) * coef[0, :C]
    ext().scale_cols(dw, coef[0])
    torch.testing.assert_close(dw.view(K, C), ref, rtol=0, atol=0)
