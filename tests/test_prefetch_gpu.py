"""Device prefetch (data/prefetch.py): the prefetched device batches are the pipeline's batches,
in order, and the end of a non-repeating pipeline / a loader error reach the training thread."""
import os

import numpy as np
import pytest
import torch

from tensorflowdistributedlearning_amd.data.pipeline import SegmentationPipeline
from tensorflowdistributedlearning_amd.data.prefetch import DevicePrefetcher

Image = pytest.importorskip("PIL.Image")


def _write(tmp, n=7, hw=24):
    rng = np.random.default_rng(0)
    imgs, masks = [], []
    for i in range(n):
        pi, pm = os.path.join(tmp, f"i{i}.png"), os.path.join(tmp, f"m{i}.png")
        Image.fromarray((rng.random((hw, hw)) * 255).astype(np.uint8), "L").save(pi)
        Image.fromarray(((rng.random((hw, hw)) > 0.6) * 255).astype(np.uint8), "L").save(pm)
        imgs.append(pi)
        masks.append(pm)
    return imgs, masks


@pytest.mark.gpu
def test_prefetched_batches_match_pipeline(tmp_path, gpu):
    imgs, masks = _write(str(tmp_path))
    kw = dict(augment=True, shuffle=True, repeat=False, seed=3, device=gpu)
    ref = [(x.cpu(), y.cpu()) for x, y in SegmentationPipeline(imgs, masks, 3, **kw)]
    pipe = SegmentationPipeline(imgs, masks, 3, **kw)
    pf = DevicePrefetcher(pipe.next_host, gpu, depth=2, cast=lambda x: x.float())
    got = []
    for x, y in pf:
        assert x.is_cuda and x.dtype == torch.float32 and y.is_cuda
        got.append((x * 1.0, y * 1.0))  # consumed on the training stream (waits on the event)
    pf.close()
    assert len(got) == len(ref) == 3  # 7 images, batch 3: the short last batch too
    with pytest.raises(StopIteration):  # (stays ended)
        next(pf)
    for (a, b), (c, d) in zip(got, ref):
        torch.testing.assert_close(a.cpu(), c.float(), rtol=0, atol=0)
        torch.testing.assert_close(b.cpu(), d, rtol=0, atol=0)


@pytest.mark.gpu
def test_prefetch_error_reaches_training_thread(gpu):
    n = [0]

    def source():
        n[0] += 1
        if n[0] > 2:
            raise RuntimeError("loader failed")
        return torch.ones(2, 4).pin_memory(), None

    pf = DevicePrefetcher(source, gpu)
    assert next(pf)[0].sum().item() == 8
    assert next(pf)[1] is None
    with pytest.raises(RuntimeError, match="loader failed"):
        next(pf)
    with pytest.raises(RuntimeError, match="loader failed"):
        next(pf)
    pf.close()
