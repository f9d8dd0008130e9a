"""Input pipelines on top of the native C++ loader (csrc/runtime/loader.cpp).

``SegmentationPipeline`` is the reference's ``Model._make_input_fn`` (model.py:285-324):
glob ``{model_dir}/{mode}/images/fold{k}/*.png`` and the parallel masks, ``shuffle_and_repeat``
(or ``repeat``), ``map(read_and_preprocess(augment))``, ``batch``, ``prefetch(2·n_gpus)`` — but the
decode/augment/batch work runs in native worker threads writing pinned host buffers, and the
H2D copy is asynchronous on the current stream.  In data-parallel runs each rank reads a disjoint
shard (images[rank::world]) with its own seed — the per-tower batches of MirroredStrategy.
``TestPipeline`` is ``Model._make_test_input`` (model.py:257-283) with a TTA transformation.
Images arrive in bf16 (the GPU compute dtype) or, with ``fp32=True``, in fp32 — normalisation,
augmentation and the Laplacian run in fp32 either way (``Model(precision="fp32")`` uses it, so the
reference-precision runs see unrounded inputs).
"""
from __future__ import annotations

import glob
import os

import torch

from .. import _native

TRANSFORMS = {"none": 0, "vertical": 1, "horizontal": 2, "transpose": 3}


def fold_files(model_dir, mode, fold):
    images = sorted(glob.glob(os.path.join(model_dir, mode, "images", f"fold{fold}", "*.png")))
    masks = sorted(glob.glob(os.path.join(model_dir, mode, "masks", f"fold{fold}", "*.png")))
    return images, masks


# what the reference's training input_fn maps: read_and_preprocess(augment, crop_probability=0)
# (model.py:315-317) with the function's other defaults (preprocessing.py:112-123)
TRAIN_AUG = {"crop_probability": 0.0}


class SegmentationPipeline:
    """``aug``: read_and_preprocess knobs for the native augmentation (horizontal_flip,
    vertical_flip, rotate_range, crop_probability, crop_min_percent, crop_max_percent,
    height_shift_range, width_shift_range, brightness_range); default :data:`TRAIN_AUG`."""

    def __init__(self, images, masks, batch_size, augment, shuffle, repeat=True, seed=0,
                 device="cpu", rank=0, world=1, threads=4, prefetch=4, channels=8, aug=None,
                 fp32=False):
        if world > 1:
            images = images[rank::world]
            masks = masks[rank::world] if masks else masks
        if masks and len(masks) != len(images):
            raise ValueError("image/mask count mismatch")
        self.n = len(images)
        self.device = torch.device(device)
        self.batch_size = batch_size
        self.ids = [os.path.splitext(os.path.basename(p))[0] for p in images]
        self._loader = _native.load().BatchLoader(
            list(images), list(masks or []), int(batch_size), bool(augment), bool(shuffle),
            bool(repeat), int(seed) * 1000 + rank, int(threads), int(prefetch), int(channels), 0,
            self.device.type == "cuda", dict(TRAIN_AUG if aug is None else aug), bool(fp32))

    def __iter__(self):
        return self

    def next_host(self):
        """The next batch as host tensors (pinned for a GPU pipeline) — data/prefetch.py copies
        them to the device on its own stream."""
        out = self._loader.next()
        if out is None:
            raise StopIteration
        x, y, ids, count = out
        if count < x.shape[0]:
            x = x[:count]
            y = y[:count] if y is not None else None
        return x, y

    def __next__(self):
        x, y = self.next_host()
        if self.device.type == "cuda":
            x = x.to(self.device, non_blocking=True)
            y = y.to(self.device, non_blocking=True) if y is not None else None
        return x, y

    @property
    def steps_per_epoch(self):
        return max(1, self.n // self.batch_size)


class TestPipeline:
    """Images only, no shuffle/repeat, optional TTA transformation; yields (x, ids)."""

    __test__ = False  # not a pytest class

    def __init__(self, images, batch_size, transformation="none", device="cpu", threads=4,
                 prefetch=4, channels=8, fp32=False):
        self.device = torch.device(device)
        self.ids = [os.path.splitext(os.path.basename(p))[0] for p in images]
        self._loader = _native.load().BatchLoader(
            list(images), [], int(batch_size), False, False, False, 0, int(threads), int(prefetch),
            int(channels), TRANSFORMS[transformation], self.device.type == "cuda", {}, bool(fp32))

    def __iter__(self):
        return self

    def __next__(self):
        out = self._loader.next()
        if out is None:
            raise StopIteration
        x, _, ids, count = out
        x = x[:count]
        ids = ids[:count]
        if self.device.type == "cuda":
            x = x.to(self.device, non_blocking=True)
        return x, [self.ids[i] for i in ids.tolist()]
