"""End-to-end training on the GPU through the HIP kernels (SURVEY §7.5 E2E tier)."""
import pytest
import torch

from tensorflowdistributedlearning_amd import models
from tensorflowdistributedlearning_amd.engine.trainer import Trainer
from tensorflowdistributedlearning_amd.ops import softmax_cross_entropy, lovasz_hinge
from tensorflowdistributedlearning_amd.data.synthetic import imagenet_batch, segmentation_batch

pytestmark = pytest.mark.gpu


def test_resnet50_steps_reduce_loss(gpu):
    torch.manual_seed(0)
    m = models.resnet50(num_classes=10)
    tr = Trainer(m, softmax_cross_entropy, gpu, "sgd", dict(lr=0.02, momentum=0.9,
                                                          weight_decay=0.0))
    x, y = imagenet_batch(16, 64, num_classes=10, device=gpu)
    losses = [float(tr.train_step(x, y)[0]) for _ in range(8)]
    assert all(l == l for l in losses), losses  # no NaN
    assert losses[-1] < losses[0], losses


def test_gpu_step_matches_cpu_reference(gpu):
    """One SGD step of a small ResNet on GPU (bf16 HIP kernels) vs the fp32 CPU oracle path."""
    torch.manual_seed(1)
    m_cpu = models.resnet18(num_classes=10)
    m_gpu = models.resnet18(num_classes=10)
    m_gpu.load_state_dict(m_cpu.state_dict())
    x, y = imagenet_batch(8, 32, num_classes=10, dtype=torch.float32)
    t_cpu = Trainer(m_cpu, softmax_cross_entropy, "cpu", "sgd", dict(lr=0.1, momentum=0.0,
                                                                     weight_decay=0.0),
                    lowp_dtype=None)
    t_gpu = Trainer(m_gpu, softmax_cross_entropy, gpu, "sgd", dict(lr=0.1, momentum=0.0,
                                                                  weight_decay=0.0))
    l_cpu, out_cpu = t_cpu.train_step(x, y)
    l_gpu, out_gpu = t_gpu.train_step(x.to(gpu, torch.bfloat16), y.to(gpu))
    assert abs(float(l_cpu) - float(l_gpu)) < 0.05 * max(1.0, abs(float(l_cpu)))
    g_cpu = t_cpu.flat.grad
    g_gpu = t_gpu.flat.grad.cpu()
    cos = torch.nn.functional.cosine_similarity(g_cpu, g_gpu, dim=0).item()
    assert cos > 0.98, cos


def test_deeplab_reference_preset_trains(gpu):
    torch.manual_seed(2)
    m = models.DeepLabResNet(model_name="m", input_shape=(101, 101))
    tr = Trainer(m, lovasz_hinge, gpu, "adam", dict(lr=1e-3))
    x, y = segmentation_batch(4, device=gpu)
    l0 = float(tr.train_step(x, y)[0])
    for _ in range(4):
        l = float(tr.train_step(x, y)[0])
    assert l == l and l < l0 + 0.5


def test_xception_forward_backward(gpu):
    torch.manual_seed(3)
    m = models.xception_41(num_classes=10)
    tr = Trainer(m, softmax_cross_entropy, gpu, "sgd", dict(lr=0.01, momentum=0.9))
    x, y = imagenet_batch(4, 64, num_classes=10, device=gpu)
    l = float(tr.train_step(x, y)[0])
    assert l == l
