"""Debug: stem BN γ gradient in a captured (frozen-BN) step vs eager — stashes the eval-mode
backward's temporaries (ops/bn.py) of the stem BN and compares them after each replay."""
import sys
import torch
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tensorflowdistributedlearning_amd import models  # noqa: E402
from tensorflowdistributedlearning_amd.engine.trainer import Trainer  # noqa: E402
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy, streams, bn as B  # noqa: E402
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch  # noqa: E402

streams.set_enabled(False)
gpu = torch.device("cuda")
torch.manual_seed(11)
nets = [models.resnet18(num_classes=10) for _ in range(2)]
nets[1].load_state_dict(nets[0].state_dict())
tr = [Trainer(n, softmax_cross_entropy, gpu, "sgd", dict(lr=0.0, momentum=0.0)) for n in nets]
for t in tr:
    t.train_mode = False
stash = {}
orig = B.deliver_grad
gam = {id(n.stem.bn.gamma): i for i, n in enumerate(nets)}


def spy(p, g=None, written=False):
    if id(p) in gam and g is not None:
        stash[gam[id(p)]] = (g, p.grad)
    return orig(p, g, written)


B.deliver_grad = spy
x, y = imagenet_batch(8, 32, num_classes=10, device=gpu)
tr[1].capture(x, y, warmup=1)
gcap = stash[1]
print("grad view is flat slice:", gcap[1].data_ptr() == tr[1].flat.grad[tr[1].flat.slice_of(nets[1].stem.bn.gamma)[0]:].data_ptr())
for s in range(3):
    tr[0].train_step(x, y)
    tr[1].replay()
    torch.cuda.synchronize()
    ge = stash[0][0]
    print(f"step {s}: temp eager vs graph-temp {(ge - gcap[0]).abs().max().item():.3e}; "
          f"graph temp vs graph p.grad {(gcap[0] - gcap[1]).abs().max().item():.3e}; "
          f"eager p.grad vs graph p.grad {(nets[0].stem.bn.gamma.grad - nets[1].stem.bn.gamma.grad).abs().max().item():.3e}")
