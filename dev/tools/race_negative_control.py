"""Negative control for tests/test_train_gpu.py's side-stream race tests: with the autograd
final-callback join disabled, reading p.grad right after backward must show a mismatch (proves
the stalled-side-stream test can detect a missing join)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from tensorflowdistributedlearning_amd import models, _native
from tensorflowdistributedlearning_amd.ops import streams
_native.load()
gpu = torch.device("cuda", 0)
torch.manual_seed(6)
m = models.resnet18(num_classes=10).to(gpu)
m.train()
for mod in m.modules():
    if mod.__class__.__name__ == "BatchNorm":
        mod.train(False)
x = torch.randn(8, 64, 64, 8, device=gpu, dtype=torch.bfloat16)
outs = []
for flag in (False, True):
    streams.set_enabled(flag)
    if flag:
        streams.join_at_backward_end = lambda dev: None  # the bug under test
    for p in m.parameters():
        p.grad = None
    if flag:
        with torch.cuda.stream(streams.side(gpu)):
            torch.cuda._sleep(20_000_000)
    m(x).float().sum().backward()
    outs.append(torch.cat([p.grad.float().flatten() for p in m.parameters() if p.grad is not None]))
torch.cuda.synchronize()
d = (outs[0] - outs[1]).abs().max().item()
print("max |serial - side(no join)| =", d, "-> race detected" if d > 0 else "-> NOT detected")
