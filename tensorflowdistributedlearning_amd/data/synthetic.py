"""Synthetic device-resident batches (BASELINE.json: "synthetic 224×224 data / random-init
weights"; there is no dataset access).  The batch is generated once on the device and re-served
every step (tf_cnn_benchmarks-style synthetic input), so input I/O is excluded from the measured
step exactly as in the reference's own synthetic-free log (Test.ipynb:210-213 times the whole
step, not the loader).  Images are NHWC with channels padded to 8 (zeros beyond the real 3 or 2)
because the conv kernels read 16-byte channel vectors.
"""
from __future__ import annotations

import torch


def imagenet_batch(batch, size=224, channels=3, pad_to=8, num_classes=1000, device="cpu",
                   dtype=torch.bfloat16, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.zeros(batch, size, size, pad_to, dtype=torch.float32)
    x[..., :channels] = torch.randn(batch, size, size, channels, generator=g)
    y = torch.randint(0, num_classes, (batch,), generator=g)
    return x.to(device=device, dtype=dtype), y.to(device)


def segmentation_batch(batch, size=(101, 101), channels=2, pad_to=8, device="cpu",
                       dtype=torch.bfloat16, seed=0):
    """TGS-shaped batch: image (normalised grey + Laplacian) and a binary mask [B,H,W,1]."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    H, W = size
    x = torch.zeros(batch, H, W, pad_to, dtype=torch.float32)
    x[..., :channels] = torch.randn(batch, H, W, channels, generator=g)
    # blobby masks: threshold a smoothed noise field
    noise = torch.randn(batch, 1, H // 4 + 1, W // 4 + 1, generator=g)
    up = torch.nn.functional.interpolate(noise, size=(H, W), mode="bilinear", align_corners=False)
    mask = (up > 0.3).float().permute(0, 2, 3, 1)
    return x.to(device=device, dtype=dtype), mask.to(device)


def repeat(batch):
    while True:
        yield batch
