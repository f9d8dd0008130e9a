"""Model structure parity (CPU): parameter counts / tensor counts / shapes vs SURVEY Appendix A,
checkpoint naming vs Appendix B, and the atrous output-stride control."""
import pytest
import torch

from tensorflowdistributedlearning_amd import models


def count(m):
    return sum(p.numel() for p in m.parameters()), len(list(m.parameters()))


def test_resnet_param_counts():
    assert count(models.resnet50())[0] == 25_557_032
    assert count(models.resnet18())[0] == 11_689_512
    assert count(models.resnet152())[0] == 60_192_808


def test_deeplab_reference_preset_matches_appendix_a():
    m = models.DeepLabResNet(model_name="model", input_shape=(101, 101))
    n, t = count(m)
    assert n == 41_814_025          # SURVEY Appendix A (exact replay of core/resnet.py)
    assert t == 208                 # 66 conv/dw weights + 24 biases + 59 BN x (gamma, beta)
    bn_moving = sum(b.numel() for name, b in m.named_buffers() if "running" in name)
    assert bn_moving == 65_632       # moving mean + variance of the 59 BN layers
    assert sum(1 for name, _ in m.named_buffers() if "running_mean" in name) == 59


def test_deeplab_shapes_and_end_points():
    m = models.DeepLabResNet(model_name="model", input_shape=(101, 101))
    x = torch.randn(2, 101, 101, 2)
    out, ep = m(x, return_end_points=True)
    assert out.shape == (2, 101, 101, 1)
    assert ep["model/resnet_v2/block4"].shape == (2, 13, 13, 1024)
    assert ep["model/resnet_v2/block1/unit_1/bottleneck_v2/conv3"].shape == (2, 26, 26, 512)
    assert ep["model/resnet_v2/block3"].shape == (2, 13, 13, 2048)


def test_deeplab_dilation_rates():
    m = models.DeepLabResNet(model_name="model")
    rates = [[u.conv2.conv.dilation[0] for u in blk] for blk in m.blocks]
    assert rates == [[1, 1, 1], [1, 1, 1, 1], [2] * 6, [4, 8, 4]]


def test_deeplab_output_stride_none_and_16():
    m = models.DeepLabResNet(model_name="m", output_stride=None, input_shape=(64, 64))
    out, ep = m(torch.randn(1, 64, 64, 2), return_end_points=True)
    assert out.shape == (1, 64, 64, 1)
    assert ep["m/resnet_v2/block4"].shape[1] == 2  # full striding: 64/32
    m16 = models.DeepLabResNet(model_name="m", output_stride=16, input_shape=(64, 64))
    _, ep = m16(torch.randn(1, 64, 64, 2), return_end_points=True)
    assert ep["m/resnet_v2/block4"].shape[1] == 4
    with pytest.raises(ValueError):
        models.DeepLabResNet(output_stride=6)


def test_deeplab_plumbing_32x32_even_input():
    """D11: decoder size derived, so even-sized inputs (TF SAME asymmetric padding) work."""
    m = models.DeepLabResNet(model_name="m", input_shape=(32, 32), n_blocks=(1, 1, 1))
    assert m(torch.randn(2, 32, 32, 2)).shape == (2, 32, 32, 1)


def test_deeplab_basic_block_variant():
    m = models.DeepLabResNet(model_name="m", block_type="basic_block", input_shape=(33, 33))
    out, ep = m(torch.randn(1, 33, 33, 2), return_end_points=True)
    assert out.shape == (1, 33, 33, 1)
    assert "m/resnet_v2/block1/unit_1/bottleneck_v2/conv2" in ep


def test_tf_names_cover_every_tensor():
    m = models.DeepLabResNet(model_name="fold_model")
    names = m.tf_names()
    sd = m.state_dict()
    assert set(names) == set(sd.keys())
    assert names["conv1_1.conv.weight"] == "fold_model/resnet_v2/conv1_1/weights"
    assert names["blocks.0.0.conv2.bn.running_var"] == \
        "fold_model/resnet_v2/block1/unit_1/bottleneck_v2/Conv/BatchNorm/moving_variance"
    assert names["assp_conv_3x3_2.depthwise.weight"] == \
        "fold_model/assp/conv/conv_3x3_2_depthwise/depthwise_weights"
    assert names["decoder_conv_3x3.bias"] == "fold_model/decoder/conv_3x3/biases"
    assert len(set(names.values())) == len(names)


def test_xception41_intended_structure():
    m = models.xception_41(num_classes=1000)
    assert len(m.units) == 3 + 8 + 2  # 8-unit middle flow (D9 fixed)
    x = torch.randn(1, 65, 65, 3)
    assert m(x).shape == (1, 1000)
    feat = models.xception_41(num_classes=0, output_stride=16)
    y = feat(torch.randn(1, 65, 65, 3))
    assert y.shape[1] == 5 and y.shape[-1] == 2048


def test_resnet_forward_shapes():
    m = models.resnet18(num_classes=10)
    assert m(torch.randn(2, 32, 32, 3)).shape == (2, 10)


@pytest.mark.parametrize("depth", [18, 50])
def test_residual_gradient_join_matches_autograd(depth):
    """ops/gradjoin.py: sharing one dx buffer between a block input's consumers gives the same
    gradients as autograd's separate sum (identity and downsample shortcuts)."""
    from tensorflowdistributedlearning_amd.ops import gradjoin
    torch.manual_seed(0)
    m = models.build(f"resnet{depth}", num_classes=5, width=8)
    x = torch.randn(2, 32, 32, 8)
    grads = []
    for enabled in (False, True):
        gradjoin.ENABLED = enabled
        try:
            m.zero_grad(set_to_none=True)
            xi = x.clone().requires_grad_(True)
            m.train()
            out = m(xi)
            out.float().pow(2).sum().backward()
            grads.append([xi.grad.clone()] + [p.grad.clone() for p in m.parameters()])
        finally:
            gradjoin.ENABLED = True
    for a, b in zip(*grads):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("flat", [False, True])
def test_deeplab_channel_padding_is_exact(flat):
    """Physical channel padding of the 258-wide block2 (defect D7; the LDS-DMA conv kernels
    need C % 8 == 0): the padded model gives the same logits, parameter gradients and moving
    statistics as the unpadded one, both through standalone parameters and through the flat
    buffers (where γ/β/bias are read from and their gradients written into the aligned slack)."""
    from tensorflowdistributedlearning_amd.models.params import FlatParams
    torch.manual_seed(0)
    kw = dict(model_name="m", input_shape=(33, 33), n_blocks=(1, 2, 1), base_depth=16)
    ref = models.DeepLabResNet(channel_align=None, **kw)
    pad = models.DeepLabResNet(channel_align=8, **kw)
    pad.load_state_dict(ref.state_dict())
    assert count(pad) == count(ref)
    assert pad.blocks[1][0].conv2.conv.padded_weight_shape() == (264, 3, 3, 264)
    assert pad.blocks[1][0].conv3.padded_weight_shape() == (1032, 1, 1, 264)
    flats = [FlatParams(m, "cpu", lowp_dtype=None) for m in (ref, pad)] if flat else None
    x = torch.randn(2, 33, 33, 2)
    res = []
    for m in (ref, pad):
        m.train()
        out, ep = m(x, return_end_points=True)
        out.float().pow(2).mean().backward()
        res.append((out, ep, [p.grad.clone() for p in m.parameters()]))
    torch.testing.assert_close(res[0][0], res[1][0], rtol=1e-4, atol=1e-5)
    assert ep["m/resnet_v2/block2"].shape[-1] == 1032
    torch.testing.assert_close(res[0][1]["m/resnet_v2/block2"], res[1][1]["m/resnet_v2/block2"],
                               rtol=1e-4, atol=1e-5)
    for (name, a), b in zip(ref.named_parameters(), res[1][2]):
        torch.testing.assert_close(res[0][2][[n for n, _ in ref.named_parameters()].index(name)],
                                   b, rtol=2e-3, atol=1e-5)
    for a, b in zip(ref.buffers(), pad.buffers()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    if flat:  # the padding slack of every flat slot is still zero
        f = flats[1]
        for p, o in zip(f.params, f.offsets):
            n = p.numel()
            end = o + (n + 63) // 64 * 64
            assert f.master[o + n:end].abs().max() == 0 if end > o + n else True
            assert f.grad[o + n:end].abs().max() == 0 if end > o + n else True


@pytest.mark.parametrize("train", [True, False])
def test_deeplab_concat_free_head_matches_cat(train):
    """The ASPP / decoder concatenations written in place (each branch's BN+ReLU and the
    upsamples store into their channel slice; backward reads slices of the concat gradient)
    compute the same logits, parameter gradients and moving statistics as the torch.cat head."""
    torch.manual_seed(3)
    kw = dict(model_name="m", input_shape=(33, 33), n_blocks=(1, 1, 1), base_depth=16)
    a = models.DeepLabResNet(**kw)
    b = models.DeepLabResNet(**kw)
    b.load_state_dict(a.state_dict())
    a.concat_free, b.concat_free = False, True
    x = torch.randn(2, 33, 33, 2)
    res = []
    for m in (a, b):
        m.train(train)
        out = m(x)
        out.float().pow(2).mean().backward()
        res.append((out, [p.grad.clone() for p in m.parameters()]))
    assert b._concat_free_ok(torch.empty(1, 5, 5, 1024))
    torch.testing.assert_close(res[0][0], res[1][0], rtol=1e-5, atol=1e-6)
    for (name, _), ga, gb in zip(a.named_parameters(), res[0][1], res[1][1]):
        torch.testing.assert_close(ga, gb, rtol=1e-4, atol=1e-6, msg=name)
    for p, q in zip(a.buffers(), b.buffers()):
        torch.testing.assert_close(p, q)


@pytest.mark.parametrize("block_type", ["bottleneck", "basic_block"])
def test_deeplab_fused_residual_units_match(block_type):
    """Units with relu(conv3 + bias + shortcut) in conv3's epilogue (plus the next pre-activation
    BN's statistics) vs the unfused units: same logits, gradients and moving statistics."""
    torch.manual_seed(4)
    kw = dict(model_name="m", input_shape=(33, 33), n_blocks=(2, 2, 1), base_depth=16,
              block_type=block_type)
    a = models.DeepLabResNet(**kw)
    b = models.DeepLabResNet(**kw)
    b.load_state_dict(a.state_dict())
    a.fuse_residual, b.fuse_residual = False, True
    x = torch.randn(2, 33, 33, 2)
    res = []
    for m in (a, b):
        m.train()
        out = m(x)
        out.float().pow(2).mean().backward()
        res.append((out, [p.grad.clone() for p in m.parameters()]))
    torch.testing.assert_close(res[0][0], res[1][0], rtol=1e-5, atol=1e-6)
    for (name, _), ga, gb in zip(a.named_parameters(), res[0][1], res[1][1]):
        torch.testing.assert_close(ga, gb, rtol=1e-4, atol=1e-6, msg=name)
    for p, q in zip(a.buffers(), b.buffers()):
        torch.testing.assert_close(p, q)


def test_xception_gradient_join_matches_autograd():
    """Xception modules: the skip's gradient and the first separable conv's depthwise dgrad meet
    in one buffer (the depthwise backward adds onto it) — same gradients as autograd's sum."""
    from tensorflowdistributedlearning_amd.models.xception import XceptionModule
    torch.manual_seed(0)
    m = models.xception_41(num_classes=5)
    x = torch.randn(2, 64, 64, 3)
    grads = []
    for enabled in (False, True):
        XceptionModule.grad_join = enabled
        try:
            m.zero_grad(set_to_none=True)
            xi = x.clone().requires_grad_(True)
            m.train()
            out = m(xi)
            out.float().pow(2).sum().backward()
            grads.append([xi.grad.clone()] + [p.grad.clone() for p in m.parameters()])
        finally:
            XceptionModule.grad_join = True
    for a, b in zip(*grads):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
