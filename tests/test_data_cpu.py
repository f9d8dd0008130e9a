"""Native data loader (csrc/runtime/loader.cpp) vs independent numpy oracles of the reference's
tf.image / tf.contrib.image semantics (preprocessing/preprocessing.py:61-216)."""
import math
import os

import numpy as np
import pytest
import torch

from tensorflowdistributedlearning_amd import _native
from tensorflowdistributedlearning_amd.preprocessing import preprocessing as P
from tensorflowdistributedlearning_amd.data.pipeline import SegmentationPipeline, TestPipeline

Image = pytest.importorskip("PIL.Image")
C = _native.load()
MEAN, STD = P.MEAN, P.STD


def _write(tmp, n=6, hw=24, seed=0):
    rng = np.random.default_rng(seed)
    imgs, masks, raw = [], [], []
    for i in range(n):
        a = (rng.random((hw, hw)) * 255).astype(np.uint8)
        m = ((rng.random((hw, hw)) > 0.6) * 255).astype(np.uint8)
        pi, pm = os.path.join(tmp, f"i{i}.png"), os.path.join(tmp, f"m{i}.png")
        Image.fromarray(a, "L").save(pi)
        Image.fromarray(m, "L").save(pm)
        imgs.append(pi)
        masks.append(pm)
        raw.append((a.astype(np.float32) / 255, m.astype(np.float32) / 255))
    return imgs, masks, raw


def np_laplace(x):
    k = np.array([[0.5, 1, 0.5], [1, -6, 1], [0.5, 1, 0.5]], np.float64)
    p = np.pad(x.astype(np.float64), 1)
    out = np.zeros_like(x, dtype=np.float64)
    for dy in range(3):
        for dx in range(3):
            out += k[dy, dx] * p[dy:dy + x.shape[0], dx:dx + x.shape[1]]
    return out


def np_transform(hflip, vflip, angle, tx, ty, H, W, crop=None):
    """tf.contrib.image.compose_transforms(hflip, vflip, angles_to_projective_transforms,
    translations_to_projective_transforms[, crop]) as a flat 8-vector; ``crop`` = (pct, left,
    top) is the reference's crop transform [pct, 0, top, 0, pct, left, 0, 0]
    (preprocessing.py:213-228)."""
    def m(t):
        return np.array([[t[0], t[1], t[2]], [t[3], t[4], t[5]], [t[6], t[7], 1.0]])
    ident = [1, 0, 0, 0, 1, 0, 0, 0]
    hf = [-1, 0, W, 0, 1, 0, 0, 0] if hflip else ident
    vf = [1, 0, 0, 0, -1, H, 0, 0] if vflip else ident
    c, s = math.cos(angle), math.sin(angle)
    xo = ((W - 1) - (c * (W - 1) - s * (H - 1))) / 2
    yo = ((H - 1) - (s * (W - 1) + c * (H - 1))) / 2
    rot = [c, -s, xo, s, c, yo, 0, 0]
    tr = [1, 0, tx, 0, 1, ty, 0, 0]
    M = m(hf) @ m(vf) @ m(rot) @ m(tr)
    if crop is not None:
        pct, left, top = crop
        M = M @ m([pct, 0, top, 0, pct, left, 0, 0])
    return (M / M[2, 2]).reshape(-1)[:8]


def np_warp(img, t, nearest):
    H, W = img.shape
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float64)
    k = t[6] * xs + t[7] * ys + 1
    ix = (t[0] * xs + t[1] * ys + t[2]) / k
    iy = (t[3] * xs + t[4] * ys + t[5]) / k

    def at(yy, xx):
        ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        return np.where(ok, img[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)], 0.0)
    if nearest:
        rnd = lambda v: np.where(v >= 0, np.floor(v + 0.5), -np.floor(-v + 0.5)).astype(np.int64)
        return at(rnd(iy), rnd(ix))
    x0, y0 = np.floor(ix).astype(np.int64), np.floor(iy).astype(np.int64)
    ax, ay = ix - x0, iy - y0
    return ((1 - ay) * ((1 - ax) * at(y0, x0) + ax * at(y0, x0 + 1))
            + ay * ((1 - ax) * at(y0 + 1, x0) + ax * at(y0 + 1, x0 + 1)))


def np_augment(img, mask, transpose, hflip, vflip, angle, tx, ty, pad, bright=0.0, crop=None):
    x = (img.astype(np.float64) - MEAN) / STD + bright
    x = np.pad(x, pad, mode="reflect")
    mk = np.pad(mask.astype(np.float64), pad, mode="reflect")
    if transpose:
        x, mk = x.T, mk.T
    H, W = x.shape
    t = np_transform(hflip, vflip, angle, tx, ty, H, W, crop)
    wi, wm = np_warp(x, t, False), np_warp(mk, t, True)
    h, w = img.shape
    return wi[pad:pad + h, pad:pad + w], wm[pad:pad + h, pad:pad + w]


def test_png_decode_matches_pil(tmp_path):
    rng = np.random.default_rng(1)
    a = (rng.random((17, 23)) * 255).astype(np.uint8)
    Image.fromarray(a, "L").save(tmp_path / "g.png")
    np.testing.assert_allclose(C.png_decode_gray(str(tmp_path / "g.png")).numpy(), a / 255.0,
                               atol=1e-6)
    a16 = (rng.random((9, 11)) * 65535).astype(np.uint16)
    Image.fromarray(a16, "I;16").save(tmp_path / "g16.png")
    np.testing.assert_allclose(C.png_decode_gray(str(tmp_path / "g16.png")).numpy(),
                               a16 / 65535.0, atol=1e-6)
    rgb = (rng.random((8, 8, 3)) * 255).astype(np.uint8)
    Image.fromarray(rgb, "RGB").save(tmp_path / "c.png")
    ref = np.asarray(Image.open(tmp_path / "c.png").convert("L"), np.float32) / 255
    np.testing.assert_allclose(C.png_decode_gray(str(tmp_path / "c.png")).numpy(), ref,
                               atol=1.5 / 255)


@pytest.mark.parametrize("hflip,vflip,angle,tx,ty", [
    (False, False, 0.0, 0.0, 0.0), (True, False, 0.1, 3.0, -2.0), (False, True, -0.17, -7.5, 4.0),
    (True, True, 0.05, 10.0, 10.0)])
def test_transform_matrix(hflip, vflip, angle, tx, ty):
    got = np.array(C.transform_matrix(hflip, vflip, angle, tx, ty, 181, 181))
    np.testing.assert_allclose(got, np_transform(hflip, vflip, angle, tx, ty, 181, 181),
                               rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("seed", range(4))
def test_augment_matches_numpy_oracle(seed):
    rng = np.random.default_rng(seed)
    img = rng.random((21, 21)).astype(np.float32)
    mask = (rng.random((21, 21)) > 0.5).astype(np.float32)
    tp, hf, vf = bool(rng.random() > 0.5), bool(rng.random() < 0.5), bool(rng.random() < 0.5)
    ang = float(rng.uniform(-0.17, 0.17))
    tx, ty = float(rng.uniform(-8, 8)), float(rng.uniform(-8, 8))
    oi, om, lap = C.augment_one(torch.from_numpy(img), torch.from_numpy(mask), tp, hf, vf, ang,
                                tx, ty, 10)
    ri, rm = np_augment(img, mask, tp, hf, vf, ang, tx, ty, 10)
    np.testing.assert_allclose(oi.numpy(), ri, atol=2e-4)
    # nearest sampling: allow a handful of exact-half rounding ties to differ
    assert (np.abs(om.numpy() - rm) > 1e-6).mean() < 0.01
    np.testing.assert_allclose(lap.numpy(), np_laplace(oi.numpy()), atol=1e-4)


@pytest.mark.parametrize("pct,left,top", [(0.9, 5.0, 12.0), (1.1, -3.0, -7.5), (1.0, 0.0, 0.0)])
def test_crop_transform_matrix(pct, left, top):
    got = np.array(C.transform_matrix(True, False, 0.1, 3.0, -2.0, 181, 181, crop=True,
                                      crop_pct=pct, crop_left=left, crop_top=top))
    np.testing.assert_allclose(got, np_transform(True, False, 0.1, 3.0, -2.0, 181, 181,
                                                 (pct, left, top)), rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("seed", range(3))
def test_augment_crop_brightness_matches_numpy_oracle(seed):
    """Random crop (scale / offset transform) and brightness delta, composed with the rest."""
    rng = np.random.default_rng(100 + seed)
    img = rng.random((21, 21)).astype(np.float32)
    mask = (rng.random((21, 21)) > 0.5).astype(np.float32)
    tp, hf, vf = bool(rng.random() > 0.5), bool(rng.random() < 0.5), bool(rng.random() < 0.5)
    ang = float(rng.uniform(-0.17, 0.17))
    tx, ty = float(rng.uniform(-8, 8)), float(rng.uniform(-8, 8))
    pct = float(rng.uniform(0.9, 1.1))
    left, top = float(rng.random() * 41 * (1 - pct)), float(rng.random() * 41 * (1 - pct))
    br = float(rng.uniform(-0.3, 0.3))
    oi, om, _ = C.augment_one(torch.from_numpy(img), torch.from_numpy(mask), tp, hf, vf, ang,
                              tx, ty, 10, brightness=br, crop=True, crop_pct=pct,
                              crop_left=left, crop_top=top)
    ri, rm = np_augment(img, mask, tp, hf, vf, ang, tx, ty, 10, br, (pct, left, top))
    np.testing.assert_allclose(oi.numpy(), ri, atol=2e-4)
    assert (np.abs(om.numpy() - rm) > 1e-6).mean() < 0.01
    # brightness only (identity geometry): the normalised image shifted by the delta
    oi, _, _ = C.augment_one(torch.from_numpy(img), None, False, False, False, 0.0, 0.0, 0.0, 10,
                             brightness=0.25)
    np.testing.assert_allclose(oi.numpy(), (img - MEAN) / STD + 0.25, atol=1e-5)


def test_loader_augmentation_options(tmp_path):
    """The loader honours read_and_preprocess's knobs (crop_probability, brightness_range, flips,
    rotation, shifts) and rejects invalid ones instead of dropping them."""
    imgs, masks, _ = _write(str(tmp_path), n=4)
    none = dict(horizontal_flip=False, vertical_flip=False, rotate_range=0.0,
                crop_probability=0.0, height_shift_range=0.0, width_shift_range=0.0)

    def first(aug):
        L = C.BatchLoader(imgs, masks, 4, True, False, False, 3, 2, 2, 8, 0, False, aug)
        x, y, _, _ = L.next()
        return x.float(), y

    base = first(none)
    crop = first(dict(none, crop_probability=1.0, crop_min_percent=0.8, crop_max_percent=0.8))
    bright = first(dict(none, brightness_range=0.5))
    assert not torch.equal(base[0], crop[0]) and not torch.equal(base[1], crop[1])
    d = (bright[0][..., 0] - base[0][..., 0]).reshape(4, -1)
    # one delta per sample (bf16 storage rounding aside), |delta| <= 0.5
    assert (d.max(1).values - d.min(1).values).abs().max() < 0.05
    assert d.abs().max() <= 0.5 + 0.05 and d.abs().mean() > 1e-3
    with pytest.raises(Exception):
        C.BatchLoader(imgs, masks, 4, True, False, False, 3, 2, 2, 8, 0, False,
                      dict(crop_probability=1.5))
    with pytest.raises(Exception):
        C.BatchLoader(imgs, masks, 4, True, False, False, 3, 2, 2, 8, 0, False,
                      dict(no_such_knob=1))


def test_read_and_preprocess_crop_and_brightness(tmp_path):
    from tensorflowdistributedlearning_amd.preprocessing import preprocessing as P
    imgs, masks, _ = _write(str(tmp_path), n=1, hw=21)
    kw = dict(horizontal_flip=False, vertical_flip=False, rotate_range=0, height_shift_range=0,
              width_shift_range=0)
    a = P.read_and_preprocess(imgs[0], masks[0], True, crop_probability=0.0, **kw,
                              rng=np.random.default_rng(0))
    b = P.read_and_preprocess(imgs[0], masks[0], True, crop_probability=1.0,
                              crop_min_percent=0.7, crop_max_percent=0.7, **kw,
                              rng=np.random.default_rng(0))
    assert not torch.equal(a[0]["images"], b[0]["images"])
    with pytest.raises(ValueError):
        P.read_and_preprocess(imgs[0], masks[0], True, crop_probability=2.0)
    with pytest.raises(ValueError):
        P.read_and_preprocess(imgs[0], masks[0], True, brightness_range=-1.0)


def test_loader_eval_batches_exact(tmp_path):
    imgs, masks, raw = _write(str(tmp_path), n=5)
    L = C.BatchLoader(imgs, masks, 2, False, False, False, 0, 3, 2, 8, 0)
    seen = []
    while True:
        out = L.next()
        if out is None:
            break
        x, y, ids, count = out
        assert x.dtype == torch.bfloat16 and x.shape == (2, 24, 24, 8)
        for j in range(count):
            i = int(ids[j])
            seen.append(i)
            a, m = raw[i]
            e = (a - MEAN) / STD
            np.testing.assert_allclose(x[j, :, :, 0].float().numpy(), e, rtol=1e-2, atol=1e-2)
            np.testing.assert_allclose(x[j, :, :, 1].float().numpy(), np_laplace(e), rtol=2e-2,
                                       atol=5e-2)
            assert torch.all(x[j, :, :, 2:] == 0)
            np.testing.assert_allclose(y[j, :, :, 0].numpy(), m, atol=1e-6)
    assert seen == [0, 1, 2, 3, 4]


def test_loader_shuffle_epochs_and_determinism(tmp_path):
    imgs, masks, _ = _write(str(tmp_path), n=6)

    def run(seed):
        L = C.BatchLoader(imgs, masks, 3, True, True, True, seed, 4, 4, 8, 0)
        out = [L.next() for _ in range(4)]
        return [o[2].tolist() for o in out], [o[0].float() for o in out]
    ids1, xs1 = run(5)
    ids2, xs2 = run(5)
    ids3, _ = run(6)
    assert ids1 == ids2 and all(torch.equal(a, b) for a, b in zip(xs1, xs2))
    assert sorted(ids1[0] + ids1[1]) == list(range(6))  # each epoch is a permutation
    assert sorted(ids1[2] + ids1[3]) == list(range(6))
    assert ids1 != ids3


def test_loader_concurrent_cache_fill_stress(tmp_path):
    # tiny dataset, many workers, repeat: concurrent first loads of the same image
    imgs, masks, _ = _write(str(tmp_path), n=2, hw=16)
    for _ in range(20):
        L = C.BatchLoader(imgs, masks, 4, True, True, True, 0, 8, 8, 8, 0)
        for _ in range(3):
            assert L.next() is not None
        del L


@pytest.mark.parametrize("kind,fn", [("vertical", lambda a: a[::-1]),
                                     ("horizontal", lambda a: a[:, ::-1]),
                                     ("transpose", lambda a: a.T), ("none", lambda a: a)])
def test_test_pipeline_tta(tmp_path, kind, fn):
    imgs, _, raw = _write(str(tmp_path), n=3)
    xs, ids = [], []
    for x, b in TestPipeline(imgs, 2, kind):
        xs.append(x)
        ids += b
    x = torch.cat(xs)
    assert ids == ["i0", "i1", "i2"]
    for j in range(3):
        e = fn((raw[j][0] - MEAN) / STD)
        np.testing.assert_allclose(x[j, :, :, 0].float().numpy(), e, rtol=1e-2, atol=1e-2)


def test_pipeline_sharding(tmp_path):
    imgs, masks, _ = _write(str(tmp_path), n=6)
    a = SegmentationPipeline(imgs, masks, 3, False, False, repeat=False, rank=0, world=2)
    b = SegmentationPipeline(imgs, masks, 3, False, False, repeat=False, rank=1, world=2)
    assert a.ids == ["i0", "i2", "i4"] and b.ids == ["i1", "i3", "i5"]
    assert len(list(a)) == 1


def test_preprocessing_helpers(tmp_path):
    imgs, masks, raw = _write(str(tmp_path), n=2)
    img, mask = P.read_image(imgs[0], masks[0])
    np.testing.assert_allclose(img["images"][..., 0].numpy(), raw[0][0], atol=1e-6)
    f, m = P.read_and_preprocess(imgs[0], masks[0], augment=False)
    e = (raw[0][0] - MEAN) / STD
    np.testing.assert_allclose(f["images"][..., 0].numpy(), e, atol=1e-5)
    np.testing.assert_allclose(f["images"][..., 1].numpy(), np_laplace(e), atol=1e-4)
    f2, m2 = P.read_and_preprocess(imgs[0], masks[0], augment=True,
                                   rng=np.random.default_rng(0))
    assert f2["images"].shape == (24, 24, 2) and m2.shape == (24, 24, 1)
    t = torch.arange(12.0).reshape(1, 3, 4, 1)
    assert torch.equal(P.single_transformation(t, "vertical")["images"], t.flip(1))
    assert torch.equal(P.single_transformation(t, "transpose")["images"], t.transpose(1, 2))
    np.testing.assert_allclose(P.laplace(e).numpy(), np_laplace(e), atol=1e-4)
    # directory layout + symlinks (preprocessing.py:61-101)
    md = str(tmp_path / "model")
    P._prepare_directory(md, 2)
    for mode in ("train", "eval"):
        for kind in ("images", "masks"):
            for k in range(2):
                assert os.path.isdir(os.path.join(md, mode, kind, f"fold{k}"))
    data = tmp_path / "data"
    (data / "images").mkdir(parents=True)
    (data / "masks").mkdir()
    os.replace(imgs[0], data / "images" / "a.png")
    os.replace(masks[0], data / "masks" / "a.png")
    P.create_symlinks(str(data), md, "train", ["a"], 1)
    assert os.path.islink(os.path.join(md, "train", "images", "fold1", "a.png"))
    P.create_symlinks(str(data), md, "train", ["a"], 1)  # idempotent


def test_native_loader_under_host_sanitizers(tmp_path):
    """ASan+UBSan and TSan builds of the loader stress harness (scripts/sanitize_native.sh)."""
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    rng = np.random.default_rng(0)
    for i in range(2):
        Image.fromarray((rng.random((16, 16)) * 255).astype(np.uint8), "L").save(tmp_path / f"i{i}.png")
        Image.fromarray(((rng.random((16, 16)) > 0.6) * 255).astype(np.uint8), "L").save(tmp_path / f"m{i}.png")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["bash", os.path.join(root, "scripts", "sanitize_native.sh"), str(tmp_path), "10"],
                       capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, TMPDIR=str(tmp_path)))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count("ok ") == 2
