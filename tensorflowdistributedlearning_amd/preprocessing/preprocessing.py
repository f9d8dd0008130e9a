"""Reference-compatible preprocessing API (preprocessing/preprocessing.py of the reference).

Function names and signatures follow the reference; tensors are NHWC ``torch`` tensors (or
numpy arrays) instead of tf.Tensors.  The batch hot path (decode → augment → Laplacian → batch)
runs in the native loader (:mod:`data.pipeline`, csrc/runtime/loader.cpp); the functions here are
the per-sample API and the fold-directory management.

* ``MEAN``, ``STD`` (preprocessing.py:7-8)
* ``make_kernel``, ``simple_conv``, ``laplace`` (:11-30)
* ``_prepare_directory`` (:33-76) — fold dirs ``{model_dir}/{train,eval}/{images,masks}/fold{k}``;
  stale links are removed (errors reported, not swallowed silently)
* ``create_symlinks`` (:79-88) — D14 simplified: links are (re)created per fold, idempotently
* ``_parse_image`` / ``read_image`` (:91-101) — real PNG decoding (D18 fixed) by the native decoder
* ``read_and_preprocess`` (:112-246), ``single_transformation[_from_jpeg|_from_matrix]`` (:104-278)
"""
from __future__ import annotations

import glob
import math
import os

import numpy as np
import torch

from .. import _native
from ..ops.dwconv import laplace as _laplace_op

MEAN = 0.47194585
STD = 0.16105755
TRAIN, EVAL = "train", "eval"   # tf.estimator.ModeKeys values


def make_kernel(a):
    """2-D array → [R, S, 1] depthwise kernel (reference makes [R, S, 1, 1])."""
    a = np.asarray(a, dtype=np.float32)
    return torch.tensor(a).reshape(a.shape[0], a.shape[1], 1)


def simple_conv(x, k):
    """Depthwise SAME conv of an [..., H, W] (or NHWC) image with kernel k [R, S, 1]."""
    from ..ops.dwconv import ref_dw_fwd
    from ..ops.conv import ConvGeom
    t = torch.as_tensor(x, dtype=torch.float32)
    squeeze = t.dim() == 2
    if squeeze:
        t = t[None, :, :, None]
    R = k.shape[0]
    p = (R - 1) // 2
    y = ref_dw_fwd(t, k.expand(R, k.shape[1], t.shape[-1]), ConvGeom((1, 1), (p, R - 1 - p, p, R - 1 - p)))
    return y[0, :, :, 0] if squeeze else y


def laplace(x):
    """2-D Laplacian (kernel [[.5,1,.5],[1,-6,1],[.5,1,.5]], SAME zero padding)."""
    t = torch.as_tensor(x, dtype=torch.float32)
    if t.dim() == 2:
        return _laplace_op(t[None, :, :, None])[0, :, :, 0]
    return _laplace_op(t)


def _prepare_directory(model_directory, n_folds=5):
    for mode in (TRAIN, EVAL):
        for kind in ("images", "masks"):
            for fold in range(n_folds):
                d = os.path.join(model_directory, mode, kind, f"fold{fold}")
                os.makedirs(d, exist_ok=True)
                for f in glob.glob(os.path.join(d, "*")):
                    try:
                        os.remove(f)
                    except OSError as e:
                        print(f"[prepare_directory] could not remove {f}: {e}")


def create_symlinks(data_dir, model_dir, mode, idx, fold):
    for x in idx:
        for kind in ("images", "masks"):
            src = os.path.abspath(os.path.join(data_dir, kind, f"{x}.png"))
            dst = os.path.join(model_dir, mode, kind, f"fold{fold}", f"{x}.png")
            if os.path.islink(dst) or os.path.exists(dst):
                if os.path.islink(dst) and os.readlink(dst) == src:
                    continue
                os.remove(dst)
            os.symlink(src, dst)


def _parse_image(filename):
    """PNG → float32 [H, W, 1] in [0, 1] (native decoder)."""
    return _native.load().png_decode_gray(str(filename)).unsqueeze(-1)


def read_image(X, y):
    return {"images": _parse_image(X)}, _parse_image(y)


def single_transformation(image, transformation="none"):
    """vertical / horizontal / transpose / none on [H, W, C] (self-inverse, so it also undoes
    the TTA transform on predictions — model.py:384-387)."""
    t = torch.as_tensor(image)
    hw = (-3, -2)
    if transformation == "vertical":
        t = t.flip(hw[0])
    elif transformation == "horizontal":
        t = t.flip(hw[1])
    elif transformation == "transpose":
        t = t.transpose(hw[0], hw[1])
    elif transformation != "none":
        raise ValueError(f"Unknown transformation {transformation}")
    return {"images": t}


def single_transformation_from_matrix(X, transformation="none"):
    return single_transformation(X, transformation)


def single_transformation_from_jpeg(X, transformation="none"):
    image = (_parse_image(X) - MEAN) / STD
    image = torch.cat([image, laplace(image[..., 0]).unsqueeze(-1)], dim=-1)
    return single_transformation(image, transformation)


def read_and_preprocess(X, y, augment=False, horizontal_flip=True, vertical_flip=True,
                        rotate_range=10, crop_probability=0.5, crop_min_percent=0.9,
                        crop_max_percent=1.1, height_shift_range=0.2, width_shift_range=0.2,
                        brightness_range=0.0, rng=None):
    """Per-sample version of the reference's augmentation (preprocessing.py:112-246; the batched
    hot path is the native loader, data/pipeline.py, with the same knobs).  Returns
    ({'images': [H,W,2]}, mask [H,W,1]).  Draw order as the reference: transpose, brightness
    (``tf.image.random_brightness``: a uniform delta in ±brightness_range added to the normalised
    image), H-flip, V-flip, rotation, shifts (per sample: D13 fixed), random crop (scale
    uniform in [crop_min_percent, crop_max_percent], offsets as the reference's crop transform,
    applied with probability ``crop_probability``)."""
    if not 0 <= crop_probability <= 1 or brightness_range < 0:
        raise ValueError("crop_probability must be in [0, 1] and brightness_range >= 0")
    rng = rng or np.random.default_rng()
    image = _parse_image(X)[..., 0].contiguous()
    mask = _parse_image(y)[..., 0].contiguous()
    C = _native.load()
    if augment:
        H = image.shape[0] + 80
        W = image.shape[1] + 80
        ang = rotate_range / 180 * math.pi
        transpose = bool(rng.uniform() > 0.5)
        bright = float(rng.uniform(-brightness_range, brightness_range)) if brightness_range > 0 \
            else 0.0
        hf = bool(horizontal_flip and rng.uniform() < 0.5)
        vf = bool(vertical_flip and rng.uniform() < 0.5)
        angle = float(rng.uniform(-ang, ang))
        tx = float(rng.uniform(-width_shift_range, width_shift_range) * H) if width_shift_range \
            else 0.0
        ty = float(rng.uniform(-height_shift_range, height_shift_range) * H) \
            if height_shift_range else 0.0
        crop, pct, left, top = False, 1.0, 0.0, 0.0
        if crop_probability > 0:
            pct = float(rng.uniform(crop_min_percent, crop_max_percent))
            left = float(rng.uniform() * W * (1 - pct))
            top = float(rng.uniform() * H * (1 - pct))
            crop = bool(rng.uniform() < crop_probability)
        img, msk, lap = C.augment_one(image, mask, transpose, hf, vf, angle, tx, ty, 40,
                                      brightness=bright, crop=crop, crop_pct=pct,
                                      crop_left=left, crop_top=top)
    else:
        img = (image - MEAN) / STD
        msk = mask
        lap = laplace(img)
    return {"images": torch.stack([img, lap], dim=-1)}, msk.unsqueeze(-1)
