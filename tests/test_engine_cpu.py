"""Engine pieces: StratifiedKFold, checkpoints, summaries, best exporter, comparator, schedule."""
import json
import os
import struct

import numpy as np
import pytest
import torch

from tensorflowdistributedlearning_amd.engine.kfold import StratifiedKFold
from tensorflowdistributedlearning_amd.engine import checkpoint as ckpt
from tensorflowdistributedlearning_amd.engine import summary as S
from tensorflowdistributedlearning_amd.engine.exporter import BestExporter, load_export
from tensorflowdistributedlearning_amd.engine.trainer import Trainer
from tensorflowdistributedlearning_amd.models.deeplab import DeepLabResNet
from tensorflowdistributedlearning_amd.ops.optim import exponential_decay
from tensorflowdistributedlearning_amd.ops.loss import lovasz_hinge
from tensorflowdistributedlearning_amd.utils import metric_comparisson, get_available_gpus


@pytest.mark.parametrize("seed", [0, 42, 7])
@pytest.mark.parametrize("n_splits", [2, 5])
def test_stratified_kfold_matches_sklearn(seed, n_splits):
    sk = pytest.importorskip("sklearn.model_selection")
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 4, size=97)
    X = np.arange(97)
    ours = list(StratifiedKFold(n_splits, True, seed).split(X, y))
    ref = list(sk.StratifiedKFold(n_splits=n_splits, shuffle=True, random_state=seed).split(X, y))
    for (a_tr, a_te), (b_tr, b_te) in zip(ours, ref):
        np.testing.assert_array_equal(a_tr, b_tr)
        np.testing.assert_array_equal(a_te, b_te)


def test_stratified_kfold_partition():
    y = np.array([0] * 10 + [1] * 5)
    folds = list(StratifiedKFold(5, True, 1).split(np.zeros(15), y))
    te = np.concatenate([t for _, t in folds])
    assert sorted(te.tolist()) == list(range(15))
    for tr, t in folds:
        assert not set(tr) & set(t)
        assert (y[t] == 1).sum() == 1


def _tiny_net():
    torch.manual_seed(0)
    return DeepLabResNet(model_name="m", in_channels=2, output_stride=8, base_depth=8,
                         input_shape=(16, 16), n_blocks=(1, 1, 1))


def test_checkpoint_roundtrip_with_adam_slots(tmp_path):
    net = _tiny_net()
    tr = Trainer(net, lambda o, y: lovasz_hinge(o, y), "cpu", optimizer="adam",
                 opt_kwargs=dict(lr=1e-3))
    x = torch.randn(2, 16, 16, 8)
    y = (torch.rand(2, 16, 16, 1) > 0.5).float()
    for _ in range(2):
        tr.train_step(x, y)
    d = str(tmp_path / "fold0")
    ckpt.save(d, 2, net, tr.optimizer, keep_max=2)
    for s in (3, 4):
        tr.train_step(x, y)
        ckpt.save(d, s, net, tr.optimizer, keep_max=2)
    # keep_max and pointer file
    files = sorted(f for f in os.listdir(d) if f.endswith(".safetensors"))
    assert files == ["model.ckpt-3.safetensors", "model.ckpt-4.safetensors"]
    assert ckpt.latest_checkpoint(d).endswith("model.ckpt-4.safetensors")
    # TF variable names in the file
    from safetensors.torch import load_file
    t = load_file(ckpt.latest_checkpoint(d))
    assert "m/resnet_v2/conv1_1/weights" in t
    assert "m/resnet_v2/conv1_1/BatchNorm/moving_mean" in t
    assert "m/resnet_v2/conv1_1/weights/Adam" in t and "m/resnet_v2/conv1_1/weights/Adam_1" in t
    assert "beta1_power" in t and int(t["global_step"][0]) == 4
    # restore into a fresh model + optimizer → identical state and identical next step
    net2 = DeepLabResNet(model_name="m", in_channels=2, output_stride=8, base_depth=8,
                         input_shape=(16, 16), n_blocks=(1, 1, 1))
    tr2 = Trainer(net2, lambda o, y: lovasz_hinge(o, y), "cpu", optimizer="adam",
                  opt_kwargs=dict(lr=1e-3))
    step = ckpt.restore(ckpt.latest_checkpoint(d), net2, tr2.optimizer, tr2.flat)
    assert step == 4 and tr2.optimizer.step_count == 4
    for (k, a), b in zip(net.state_dict().items(), net2.state_dict().values()):
        assert torch.equal(a, b), k
    torch.testing.assert_close(tr.optimizer.m, tr2.optimizer.m)
    tr.train_step(x, y)
    tr2.train_step(x, y)
    torch.testing.assert_close(tr.flat.master, tr2.flat.master, rtol=1e-5, atol=1e-6)
    # a checkpoint of another preset (different depth) is refused, not half-loaded
    net3 = DeepLabResNet(model_name="m", in_channels=2, output_stride=8, base_depth=8,
                         input_shape=(16, 16), n_blocks=(1, 2, 1))
    before = {k: v.clone() for k, v in net3.state_dict().items()}
    with pytest.raises(ckpt.CheckpointMismatchError, match="missing"):
        ckpt.restore(ckpt.latest_checkpoint(d), net3)
    assert all(torch.equal(before[k], v) for k, v in net3.state_dict().items())
    with pytest.warns(UserWarning, match="partial restore"):
        ckpt.restore(ckpt.latest_checkpoint(d), net3, strict=False)


def test_crc32c_and_tfrecord_framing(tmp_path):
    assert S.crc32c(b"123456789") == 0xE3069283
    assert S.crc32c(b"") == 0
    w = S.SummaryWriter(str(tmp_path))
    w.scalar("loss/lovasz_loss", 1.25, 20)
    w.scalars({"metrics/mean_iou": 0.5, "metrics/mean_acc": 0.75}, 40)
    w.image("train/train_image", np.linspace(0, 1, 12).reshape(3, 4), 40)
    w.close()
    ev = [f for f in os.listdir(tmp_path) if f.startswith("events.out.tfevents")]
    recs = list(S.read_tfrecords(os.path.join(tmp_path, ev[0])))
    assert len(recs) == 5
    assert b"brain.Event:2" in recs[0]
    assert b"loss/lovasz_loss" in recs[1] and struct.pack("<f", 1.25) in recs[1]
    assert b"\x89PNG" in recs[4]
    lines = [json.loads(l) for l in open(os.path.join(tmp_path, "scalars.jsonl"))]
    assert [l["tag"] for l in lines] == ["loss/lovasz_loss", "metrics/mean_iou",
                                        "metrics/mean_acc"]
    assert lines[1]["step"] == 40


def test_png_encoder_decodes():
    Image = pytest.importorskip("PIL.Image")
    import io
    a = np.random.default_rng(0).random((7, 5))
    im = np.asarray(Image.open(io.BytesIO(S.encode_png_gray(a))))
    np.testing.assert_array_equal(im, (a * 255 + 0.5).astype(np.uint8))


def test_metric_comparisson_fixed_semantics():
    # D4 fixed: True when the *current* result is better
    assert metric_comparisson({"iou": 0.5}, {"iou": 0.6}, "iou", True)
    assert not metric_comparisson({"iou": 0.6}, {"iou": 0.5}, "iou", True)
    assert metric_comparisson({"loss": 0.6}, {"loss": 0.5}, greater_is_better=False)
    assert not metric_comparisson({"loss": 0.6}, {"loss": 0.5})  # default greater_is_better
    with pytest.raises(ValueError):
        metric_comparisson({}, {"loss": 1.0})
    with pytest.raises(ValueError):
        metric_comparisson({"loss": 1.0}, {"x": 1.0})
    assert isinstance(get_available_gpus(), list)


def test_best_exporter(tmp_path):
    import functools
    net = _tiny_net()
    cmp = functools.partial(metric_comparisson, key="metrics/mean_iou", greater_is_better=True)
    ex = BestExporter(str(tmp_path / "export"), cmp, exports_to_keep=2,
                      serving_shape=[None, 16, 16, 2])
    assert ex.maybe_export(net, {"metrics/mean_iou": 0.3}, 1) is not None
    assert ex.maybe_export(net, {"metrics/mean_iou": 0.2}, 2) is None
    import time
    time.sleep(0.01)
    assert ex.maybe_export(net, {"metrics/mean_iou": 0.4}, 3) is not None
    time.sleep(0.01)
    p = ex.maybe_export(net, {"metrics/mean_iou": 0.5}, 4)
    bundles = sorted(os.listdir(ex.dir))
    assert len(bundles) == 2
    # a fresh exporter picks up the best result on disk
    ex2 = BestExporter(str(tmp_path / "export"), cmp, exports_to_keep=2)
    assert ex2.best["metrics/mean_iou"] == 0.5
    net2 = _tiny_net()
    with torch.no_grad():
        for v in net2.parameters():
            v.zero_()
    load_export(p, net2)
    for a, b in zip(net.state_dict().values(), net2.state_dict().values()):
        assert torch.equal(a, b)


def test_exponential_decay():
    assert exponential_decay(1e-3, 0) == 1e-3
    assert abs(exponential_decay(1e-3, 10000) - 5e-4) < 1e-15
    assert abs(exponential_decay(1e-3, 5000) - 1e-3 * 0.5 ** 0.5) < 1e-15
    assert exponential_decay(1e-3, 15000, staircase=True) == 5e-4


def test_weight_decay_exemptions_survive_deepcopy():
    """BN γ/β and biases are exempt from weight decay (models/params.FlatParams).  The exemption is
    a module-level declaration (``no_decay_params``): copy.deepcopy drops attributes set on a
    Parameter, and a deep-copied model used to train with decay on its BN parameters."""
    import copy
    from tensorflowdistributedlearning_amd import models
    from tensorflowdistributedlearning_amd.models.params import FlatParams
    m = models.resnet18(num_classes=10)
    a = FlatParams(m, "cpu", lowp_dtype=None).decay_flags
    b = FlatParams(copy.deepcopy(models.resnet18(num_classes=10)), "cpu", lowp_dtype=None).decay_flags
    assert torch.equal(a, b)
    assert 0 < int(a.sum()) < a.numel()  # conv weights decay, BN parameters do not
