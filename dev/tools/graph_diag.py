"""Where does a captured training step leave the eager trajectory?  Deterministic mode, ResNet-50
b8 64px, SGD-momentum: eager on the default stream, eager on a side stream, and HIP-graph captures
with 1 / 3 warm-up steps, with and without the side-stream weight gradients inside the graph."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflowdistributedlearning_amd import models  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy, streams  # noqa: E402
from tensorflowdistributedlearning_amd.ops.common import ext  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch  # noqa: E402

gpu = torch.device("cuda", 0)
torch.manual_seed(5)
x, y = imagenet_batch(8, 64, device=gpu)
m0 = models.resnet50(num_classes=1000)
opt = dict(lr=0.01, momentum=0.9)
ext().det_set(1)
arch = sys.argv[1] if len(sys.argv) > 1 else "resnet50"


def eager(n, stream=None):
    t = Trainer(copy.deepcopy(m0), softmax_cross_entropy, gpu, "sgd", opt)
    if stream is None:
        return [float(t.train_step(x, y)[0]) for _ in range(n)]
    with torch.cuda.stream(stream):
        out = [t.train_step(x, y)[0] for _ in range(n)]
    torch.cuda.synchronize()
    return [float(v) for v in out]


def graph(warm, n):
    t = Trainer(copy.deepcopy(m0), softmax_cross_entropy, gpu, "sgd", opt)
    t.capture(x, y, warmup=warm)
    out = [float(t.warmup_out[0])] + [float(t.replay()[0]) for _ in range(n)]
    return out


ref = eager(5)
print("eager default     ", ref, flush=True)
print("eager default (2) ", eager(5), flush=True)
print("eager side stream ", eager(5, torch.cuda.Stream(gpu)), flush=True)
print("graph warmup 1    ", graph(1, 4), "(first = the eager warm-up step)", flush=True)
print("graph warmup 3    ", graph(3, 2), "(first = warm-up step 3)", flush=True)
streams.IN_GRAPH = False
print("graph wu1 no side ", graph(1, 4), flush=True)
streams.IN_GRAPH = True
streams.set_enabled(False)
print("eager no side     ", eager(5), flush=True)
print("graph wu1 no side stream at all", graph(1, 4), flush=True)
