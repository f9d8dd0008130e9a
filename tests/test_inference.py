"""Inference path: eval-mode BatchNorm folded into the producing conv (layers.ConvBN) and into
the depthwise conv of Xception's separable convs (xception.SeparableConvBN).  CPU: the folded
forward equals the unfolded conv + BN-apply forward (fp32 oracle kernels) on ResNet, Xception and
the reference DeepLab preset, and the fold cache follows train()/eval() switches and checkpoint
loads.  GPU: the folded bf16 forward vs the unfolded bf16 forward and vs the CPU fp32 oracle."""
import copy

import pytest
import torch

from tensorflowdistributedlearning_amd import models
from tensorflowdistributedlearning_amd.models.layers import BatchNorm
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch, segmentation_batch


def _randomize_bn(net, seed=0):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, BatchNorm):
                c = m.c
                m.running_mean.copy_(torch.rand(c, generator=g) * 0.4 - 0.2)
                m.running_var.copy_(torch.rand(c, generator=g) * 1.5 + 0.5)
                if m.gamma is not None:
                    m.gamma.copy_(torch.rand(c, generator=g) + 0.5)
                m.beta.copy_(torch.rand(c, generator=g) * 0.4 - 0.2)
    return net


def _eval(net, x, fold, monkeypatch):
    monkeypatch.setenv("TDL_BN_FOLD", "1" if fold else "0")
    net.eval()
    with torch.no_grad():
        out = net(x)
    return out[0] if isinstance(out, tuple) else out


CASES = {
    "resnet18": (lambda: models.build("resnet18", num_classes=10, width=8),
                 lambda: imagenet_batch(2, 32, num_classes=10, dtype=torch.float32)[0]),
    "resnet50": (lambda: models.build("resnet50", num_classes=10),
                 lambda: imagenet_batch(2, 32, num_classes=10, dtype=torch.float32)[0]),
    "xception41": (lambda: models.xception_41(num_classes=10),
                   lambda: imagenet_batch(2, 48, num_classes=10, dtype=torch.float32)[0]),
    "deeplab": (lambda: models.DeepLabResNet(model_name="m", input_shape=(65, 65)),
                lambda: segmentation_batch(2, size=(65, 65), dtype=torch.float32)[0]),
}


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", list(CASES))
def test_bn_fold_matches_unfolded_cpu(name, monkeypatch):
    build, data = CASES[name]
    torch.manual_seed(3)
    net = _randomize_bn(build())
    x = data()
    ref = _eval(net, x, False, monkeypatch)
    got = _eval(net, x, True, monkeypatch)
    assert got.shape == ref.shape
    err = (got - ref).abs().max().item()
    assert err < 1e-4 * max(1.0, ref.abs().max().item()), err


def test_bn_fold_cache_follows_mode_switch_and_load(monkeypatch):
    torch.manual_seed(4)
    net = _randomize_bn(models.build("resnet18", num_classes=10, width=8))
    x = imagenet_batch(2, 32, num_classes=10, dtype=torch.float32)[0]
    a = _eval(net, x, True, monkeypatch)
    # the moving statistics change (as a training step would change them) → the next eval()
    # refolds
    net.train()
    _randomize_bn(net, seed=9)
    b = _eval(net, x, True, monkeypatch)
    assert not torch.allclose(a, b)
    assert torch.allclose(b, _eval(net, x, False, monkeypatch), atol=1e-4, rtol=1e-4)
    # a checkpoint load in eval mode refolds too
    other = _randomize_bn(models.build("resnet18", num_classes=10, width=8), seed=11)
    net.load_state_dict(other.state_dict())
    c = _eval(net, x, True, monkeypatch)
    assert torch.allclose(c, _eval(other, x, False, monkeypatch), atol=1e-4, rtol=1e-4)


def test_bn_fold_only_without_autograd(monkeypatch):
    """eval mode WITH autograd (input gradients, e.g. saliency) keeps the unfolded, differentiable
    path."""
    torch.manual_seed(5)
    net = _randomize_bn(models.build("resnet18", num_classes=10, width=8))
    monkeypatch.setenv("TDL_BN_FOLD", "1")
    net.eval()
    x = imagenet_batch(2, 32, num_classes=10, dtype=torch.float32)[0].requires_grad_(True)
    net(x).sum().backward()
    assert x.grad is not None and torch.isfinite(x.grad).all()


# ---------------------------------------------------------------------------------------------
def _gpu_pair(build, x_cpu, gpu):
    """The same bf16-rounded weights on the GPU (flat bf16 compute copies via the Trainer) and
    on the CPU fp32 oracle."""
    from tensorflowdistributedlearning_amd.engine.trainer import Trainer
    from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy
    torch.manual_seed(7)
    net = _randomize_bn(build())
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    cpu = copy.deepcopy(net)
    Trainer(net, softmax_cross_entropy, gpu, "sgd", dict(lr=0.0))
    return net, cpu


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", ["resnet50", "xception41", "deeplab"])
def test_bn_fold_gpu_matches_unfolded_and_oracle(gpu, name, monkeypatch):
    build, data = CASES[name]
    x = data()
    net, cpu = _gpu_pair(build, x, gpu)
    xg = x.to(gpu, torch.bfloat16)
    f = _eval(net, xg, True, monkeypatch).float().cpu()
    u = _eval(net, xg, False, monkeypatch).float().cpu()
    o = _eval(cpu, x.to(torch.bfloat16).float(), False, monkeypatch).float()
    cs = torch.nn.functional.cosine_similarity
    c_fu = cs(f.flatten(), u.flatten(), dim=0).item()
    c_fo = cs(f.flatten(), o.flatten(), dim=0).item()
    c_uo = cs(u.flatten(), o.flatten(), dim=0).item()
    print(f"{name}: folded~unfolded {c_fu:.5f} folded~oracle {c_fo:.5f} unfolded~oracle {c_uo:.5f}")
    assert torch.isfinite(f).all()
    assert c_fu > 0.995 and c_fo > 0.99, (c_fu, c_fo)
    assert c_fo > c_uo - 0.005  # folding costs no accuracy against the fp32 oracle


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bn_fold_gpu_graph_replay(gpu, monkeypatch):
    """The folded inference forward captures as one HIP graph and replays bit-identically."""
    build, data = CASES["resnet50"]
    net, _ = _gpu_pair(build, data(), gpu)
    monkeypatch.setenv("TDL_BN_FOLD", "1")
    net.eval()
    x = imagenet_batch(8, 64, num_classes=10, device=gpu)[0]
    with torch.no_grad():
        ref = net(x)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            net(x)  # warm-up on the capture stream (fold cache, kernel attributes)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = net(x)
        g.replay()
        torch.cuda.synchronize()
    assert torch.equal(out, ref)
