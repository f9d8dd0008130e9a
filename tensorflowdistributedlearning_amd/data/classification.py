"""Classification inputs for the north-star workloads trained through ``Model`` (SURVEY §2.7:
ImageNet-shaped ResNet-18/50/152 and Xception-41 with softmax cross-entropy).

The reference reaches its classifier through the same ``Model``/``resnet_model`` path
(/root/reference/core/resnet.py:246-256 logits head) but ships no classification dataset, and this
environment has no dataset access, so two sources exist:

* :class:`SyntheticImages` — a *learnable* synthetic dataset keyed by sample id: every class has a
  fixed low-resolution template (per channel, 8×8, bilinearly upsampled to the image size) and a
  sample is ``template[label] + noise``.  Noise is drawn per batch from a generator seeded by
  ``(seed, epoch, batch index, rank)``, so a run is reproducible and a resumed run sees the same
  stream as an uninterrupted one.  Top-1 accuracy therefore measures real learning (tests use it).
* :class:`ArrayImages` — an in-memory image array ``[N, H, W, C]`` (uint8 or float) with
  per-channel mean/std normalisation.

:class:`ClassificationPipeline` is the classification twin of ``SegmentationPipeline``
(data/pipeline.py): shuffle-and-repeat or one ordered pass, a disjoint shard per data-parallel rank
(the per-tower batches of MirroredStrategy), NHWC batches with channels zero-padded to 8 (the conv
kernels read 16-byte channel vectors), delivered on the training device.
"""
from __future__ import annotations

import numpy as np
import torch


class SyntheticImages:
    def __init__(self, num_classes, image_size, channels=3, seed=0, noise=1.0, signal=1.0):
        self.num_classes = int(num_classes)
        self.image_size = int(image_size)
        self.channels = int(channels)
        self.seed = int(seed)
        self.noise = float(noise)
        g = torch.Generator().manual_seed(self.seed * 7919 + 17)
        self.templates = torch.randn(self.num_classes, self.channels, 8, 8, generator=g) * signal
        self._dev = {}

    def batch(self, ids, labels, device, dtype, gen_seed):
        """Images for ``ids`` (their labels given) as [B, S, S, C] fp32 on ``device``."""
        device = torch.device(device)
        t = self._dev.get(device)
        if t is None:
            t = self._dev[device] = self.templates.to(device)
        lab = torch.as_tensor(labels, device=device, dtype=torch.long)
        s = self.image_size
        base = torch.nn.functional.interpolate(t[lab], size=(s, s), mode="bilinear",
                                               align_corners=False)
        g = torch.Generator(device=device).manual_seed(int(gen_seed) & 0x7FFFFFFFFFFFFFFF)
        x = base + self.noise * torch.randn(base.shape, generator=g, device=device)
        return x.permute(0, 2, 3, 1)


class ArrayImages:
    def __init__(self, images, mean=None, std=None):
        a = np.asarray(images)
        if a.ndim == 3:
            a = a[..., None]
        if a.ndim != 4:
            raise ValueError(f"expected images [N, H, W, C], got shape {a.shape}")
        self.images = a
        self.channels = a.shape[-1]
        self.image_size = a.shape[1]
        scale = 255.0 if a.dtype == np.uint8 else 1.0
        self.scale = scale
        if mean is None or std is None:
            m, s = self._channel_stats(a, scale)
            mean = m if mean is None else mean
            std = s if std is None else std
        self.mean = np.asarray(mean, dtype=np.float32)
        self.std = np.asarray(std, dtype=np.float32)

    @staticmethod
    def _channel_stats(a, scale, chunk_bytes=64 << 20):
        """Per-channel mean / std (+1e-6) accumulated over chunks of images (float64 sums of one
        chunk at a time: a uint8 dataset is never copied whole at 8 bytes per element)."""
        C = a.shape[-1]
        per_img = max(1, int(np.prod(a.shape[1:])))
        step = max(1, chunk_bytes // (8 * per_img))
        s1 = np.zeros(C, np.float64)
        s2 = np.zeros(C, np.float64)
        n = 0
        for i in range(0, a.shape[0], step):
            c = a[i:i + step].reshape(-1, C).astype(np.float64) / scale
            s1 += c.sum(0)
            s2 += (c * c).sum(0)
            n += c.shape[0]
        mean = s1 / max(n, 1)
        var = np.maximum(s2 / max(n, 1) - mean * mean, 0.0)
        return mean, np.sqrt(var) + 1e-6

    def batch(self, ids, labels, device, dtype, gen_seed):
        """The raw samples cross to the device as stored (uint8: a quarter of the fp32 bytes, from
        pinned memory, asynchronously) and are normalised there — host fp32 normalisation of a
        299² batch cost tens of ms per step on the training thread."""
        dev = torch.device(device)
        raw = torch.from_numpy(np.ascontiguousarray(self.images[np.asarray(ids)]))
        if dev.type == "cuda":
            raw = raw.pin_memory().to(dev, non_blocking=True)
        st = self.__dict__.setdefault("_stats", {})
        if dev not in st:
            st[dev] = (torch.from_numpy(self.mean).to(dev), torch.from_numpy(self.std).to(dev))
        mean, std = st[dev]
        x = raw.float()
        if self.scale != 1.0:
            x = x / self.scale
        return (x - mean) / std


class ClassificationPipeline:
    """Yields ``(x [B, S, S, pad_to] in dtype, y [B] int64)`` for the samples ``ids`` of a fold.

    ``repeat``: an endless shuffled stream (training); otherwise one ordered pass whose last
    batch may be short (evaluation).  ``world > 1``: rank ``rank`` reads ``ids[rank::world]``."""

    def __init__(self, source, ids, labels, batch_size, shuffle=True, repeat=True, seed=0,
                 device="cpu", rank=0, world=1, dtype=torch.bfloat16, pad_to=8, start_step=0):
        ids = np.asarray(ids)
        labels = np.asarray(labels)
        if len(ids) != len(labels):
            raise ValueError("ids / labels length mismatch")
        if world > 1:
            ids, labels = ids[rank::world], labels[rank::world]
        if repeat and len(ids) < batch_size:
            raise ValueError(f"{len(ids)} samples per rank < batch size {batch_size}")
        self.source = source
        self.ids, self.labels = ids, labels
        self.batch_size = int(batch_size)
        self.shuffle, self.repeat = shuffle, repeat
        self.seed, self.rank = int(seed), int(rank)
        self.device = torch.device(device)
        self.dtype = dtype
        self.pad_to = max(pad_to, source.channels)
        self.per_epoch = len(ids) // self.batch_size if repeat else -(-len(ids) // self.batch_size)
        # resume: continue the stream where an uninterrupted run would be after start_step batches
        self.step = int(start_step)

    @property
    def steps_per_epoch(self):
        return max(1, self.per_epoch)

    def _order(self, epoch):
        if not self.shuffle:
            return np.arange(len(self.ids))
        return np.random.default_rng((self.seed, epoch, self.rank)).permutation(len(self.ids))

    def __iter__(self):
        return self

    def __next__(self):
        if not self.repeat and self.step >= self.per_epoch:
            raise StopIteration
        epoch, b = divmod(self.step, max(self.per_epoch, 1))
        sel = self._order(epoch)[b * self.batch_size:(b + 1) * self.batch_size]
        self.step += 1
        ids, lab = self.ids[sel], self.labels[sel]
        x = self.source.batch(ids, lab, self.device, self.dtype,
                              gen_seed=hash((self.seed, epoch, b, self.rank)))
        if x.shape[-1] < self.pad_to:
            x = torch.nn.functional.pad(x, (0, self.pad_to - x.shape[-1]))
        y = torch.as_tensor(lab, dtype=torch.long).to(self.device, non_blocking=True)
        return x.to(self.dtype).contiguous(), y
