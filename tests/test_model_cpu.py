"""End-to-end ``Model`` (k-fold train → checkpoints → summaries → best export → predict) on a tiny
synthetic PNG dataset, on the CPU (reference model.py:138-255; SURVEY §4 test strategy)."""
import json
import os

import numpy as np
import pytest
import torch

from tensorflowdistributedlearning_amd.model import Model
from tensorflowdistributedlearning_amd.engine import checkpoint as ckpt
from tensorflowdistributedlearning_amd.engine.summary import read_tfrecords

PIL = pytest.importorskip("PIL.Image")

SMALL = dict(input_shape=(32, 32), n_blocks=(1, 1, 1), base_depth=16, output_stride=8,
             device="cpu", save_checkpoints_steps=2, save_summary_steps=1, loader_threads=2)


def _dataset(root, n=8, hw=32, seed=0):
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, "images"))
    os.makedirs(os.path.join(root, "masks"))
    ids, cov = [], []
    for i in range(n):
        img = (rng.random((hw, hw)) * 255).astype(np.uint8)
        m = np.zeros((hw, hw), np.uint8)
        if i % 2:
            r = rng.integers(4, 12)
            m[hw // 2 - r: hw // 2 + r, hw // 2 - r: hw // 2 + r] = 255
            img[m > 0] = np.clip(img[m > 0].astype(int) + 80, 0, 255)
        name = f"s{i:03d}"
        PIL.fromarray(img, "L").save(os.path.join(root, "images", name + ".png"))
        PIL.fromarray(m, "L").save(os.path.join(root, "masks", name + ".png"))
        ids.append(name)
        cov.append(i % 2)
    return np.array(ids), np.array(cov)


def test_model_kfold_train_export_predict(tmp_path):
    X, y = _dataset(str(tmp_path / "data"))
    md = str(tmp_path / "runs" / "tiny")
    m = Model(md, str(tmp_path / "data"), n_gpus=1, n_fold=2, save_best=2, lr=1e-3, **SMALL)
    with pytest.raises(ValueError):
        _ = m.params
    res = m.train(X, y, batch_size=2, steps=3)
    assert len(res) == 2
    assert m.params > 0
    for i in range(2):
        fd = os.path.join(md, f"fold{i}")
        # checkpoints every 2 steps + the final one, TF-style pointer file
        assert os.path.exists(os.path.join(fd, "model.ckpt-2.safetensors"))
        assert ckpt.latest_checkpoint(fd).endswith("model.ckpt-3.safetensors")
        with open(os.path.join(fd, "checkpoint")) as f:
            assert 'model_checkpoint_path: "model.ckpt-3"' in f.read()
        ev = res[i]["eval"]
        for k in ("metrics/mean_iou", "metrics/mean_acc", "loss/lovasz_loss"):
            assert k in ev and np.isfinite(ev[k])
        # summaries (TFRecord event files)
        tr = [f for f in os.listdir(os.path.join(fd, "train")) if f.startswith("events.out")]
        assert tr
        recs = list(read_tfrecords(os.path.join(fd, "train", tr[0])))
        assert len(recs) >= 4  # file_version + 3 steps
        # best exporter bundle
        ed = os.path.join(fd, "export", "best_exporter")
        bundles = [d for d in os.listdir(ed) if d.isdigit()]
        assert 1 <= len(bundles) <= 2
        with open(os.path.join(ed, bundles[-1], "config.json")) as f:
            cfg = json.load(f)
        assert cfg["signature"]["inputs"]["images"] == [None, 32, 32, 2]
    # symlinked split: disjoint train/eval, union = all ids
    tr = set(os.listdir(os.path.join(md, "train", "images", "fold0")))
    ev = set(os.listdir(os.path.join(md, "eval", "images", "fold0")))
    assert not tr & ev and len(tr | ev) == len(X)

    # resume: Estimator semantics — steps is the global max step
    res2 = m.train(X, y, batch_size=2, steps=4)
    assert res2[0]["steps"] == 4
    assert ckpt.latest_checkpoint(os.path.join(md, "fold0")).endswith("model.ckpt-4.safetensors")

    out = m.predict(os.path.join(str(tmp_path / "data"), "images"), batch_size=3, tti=True)
    assert out["probabilities"].shape == (len(X), 32, 32)
    assert out["mask"].dtype == np.uint8
    assert sorted(out["ids"]) == sorted(X.tolist())
    assert np.all((out["probabilities"] >= 0) & (out["probabilities"] <= 1))


def test_model_rejects_bad_args(tmp_path):
    with pytest.raises(ValueError):
        Model(str(tmp_path / "m"), str(tmp_path), data_format="NWHC")
    m = Model(str(tmp_path / "m"), str(tmp_path), n_gpus=2, n_fold=2, **SMALL)
    with pytest.raises(ValueError):
        m.train(np.array(["a", "b", "c", "d"]), np.array([0, 1, 0, 1]), batch_size=3, steps=1)


def test_model_batch_norm_decay_kwarg(tmp_path):
    # D2 fixed: batch_norm_decay kwarg is honoured (the reference read weight_decay)
    m = Model(str(tmp_path / "m"), str(tmp_path), batch_norm_decay=0.5, weight_decay=0.1, **SMALL)
    assert m.batch_norm_decay == 0.5
    net = m.build_network()
    assert abs(net.postnorm.bn.decay - 0.5) < 1e-12


def test_model_data_parallel_gloo(tmp_path):
    """n_gpus=2 on the host: two gloo ranks, sharded loader, all-reduced grads + eval sums."""
    X, y = _dataset(str(tmp_path / "data"), n=8, seed=1)
    md = str(tmp_path / "runs" / "dp")
    m = Model(md, str(tmp_path / "data"), n_gpus=2, n_fold=2, save_best=1, **SMALL)
    res = m.train(X, y, batch_size=4, steps=2)
    assert len(res) == 2 and all(r["steps"] == 2 for r in res)
    assert ckpt.latest_checkpoint(os.path.join(md, "fold1")).endswith("model.ckpt-2.safetensors")


@pytest.mark.gpu
def test_model_train_predict_on_gpu(tmp_path, gpu):
    """Same k-fold flow on the GPU at the reference's 101×101 input (native kernels + loader)."""
    X, y = _dataset(str(tmp_path / "data"), n=8, hw=101, seed=3)
    md = str(tmp_path / "runs" / "gpu")
    kw = dict(SMALL, device=None, input_shape=(101, 101), save_checkpoints_steps=3)
    m = Model(md, str(tmp_path / "data"), n_gpus=1, n_fold=2, save_best=1, **kw)
    res = m.train(X, y, batch_size=4, steps=3)
    assert all(np.isfinite(r["eval"]["loss/lovasz_loss"]) for r in res)
    out = m.predict(os.path.join(str(tmp_path / "data"), "images"), batch_size=4, tti=True)
    assert out["probabilities"].shape == (8, 101, 101)


@pytest.mark.gpu
def test_model_train_predict_fp32_on_gpu(tmp_path, gpu):
    """``Model(precision="fp32")``: the reference's own precision — fp32 master weights read
    directly by the fp32 kernels (no bf16 compute copy), fp32 activations end to end."""
    X, y = _dataset(str(tmp_path / "data"), n=8, hw=101, seed=4)
    md = str(tmp_path / "runs" / "gpu32")
    kw = dict(SMALL, device=None, input_shape=(101, 101), save_checkpoints_steps=3)
    m = Model(md, str(tmp_path / "data"), n_gpus=1, n_fold=2, save_best=1, precision="fp32", **kw)
    res = m.train(X, y, batch_size=4, steps=3)
    assert all(np.isfinite(r["eval"]["loss/lovasz_loss"]) for r in res)
    out = m.predict(os.path.join(str(tmp_path / "data"), "images"), batch_size=4)
    assert out["probabilities"].shape == (8, 101, 101)


def test_model_precision_option(tmp_path):
    with pytest.raises(ValueError):
        Model(str(tmp_path / "m"), str(tmp_path), precision="fp16", **SMALL)
    m = Model(str(tmp_path / "m"), str(tmp_path), precision="fp32", **SMALL)
    assert m.config()["precision"] == "fp32"
    assert m._cast(torch.zeros(2, dtype=torch.bfloat16)).dtype == torch.float32


def test_model_reference_surface_helpers(tmp_path):
    """build_model_fn_optimizer / _make_input_fn / _make_test_input (model.py:257-505)."""
    X, y = _dataset(str(tmp_path / "data"), n=4)
    md = str(tmp_path / "runs" / "api")
    m = Model(md, str(tmp_path / "data"), n_gpus=1, n_fold=2, **SMALL)
    from tensorflowdistributedlearning_amd.preprocessing.preprocessing import create_symlinks
    create_symlinks(str(tmp_path / "data"), md, "train", X[:2], 0)
    spec = m.build_model_fn_optimizer()("train", device="cpu")
    it = m._make_input_fn("train", 0, 2, augment=True, shuffle=True)()
    xb, yb = next(it)
    loss, out = spec["trainer"].train_step(xb, yb)
    assert out.shape == (2, 32, 32, 1) and torch.isfinite(loss)
    ev = m.build_model_fn_optimizer()("predict", device="cpu")
    xs, ids = next(iter(m._make_test_input(3, str(tmp_path / "data" / "images"), "vertical")()))
    assert xs.shape[0] == 3 and len(ids) == 3
    assert ev["network"](xs).shape == (3, 32, 32, 1)
