"""End-to-end ResNet training on the GPU through dtg's kernels."""
import pytest
import torch

import dtg  # noqa: F401
from dtg import ops
from dtg.models import resnet
from dtg.parallel import FlatParams, DataParallel
from dtg.optim import FusedSGD

pytestmark = pytest.mark.gpu


def test_resnet_tiny_loss_decreases():
    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = resnet.resnet18_like_tiny(10).to(dev).to(memory_format=torch.channels_last)
    flat = FlatParams(model)
    dp = DataParallel(flat)
    opt = FusedSGD(flat, lr=0.05, momentum=0.9)
    x, y = resnet.synthetic_batch(32, dev, torch.bfloat16, 32, 10, seed=1)
    losses = []
    for _ in range(30):
        loss = ops.softmax_cross_entropy(model(x), y)
        loss.backward()
        dp.finish()
        opt.step(dp.grad_scale)
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < 0.5 * losses[0], losses


def test_resnet50_step_matches_reference_direction():
    """One ResNet-50 step on a small batch: finite loss, grads flow into the flat buffer."""
    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = resnet.resnet50().to(dev).to(memory_format=torch.channels_last)
    flat = FlatParams(model)
    x, y = resnet.synthetic_batch(4, dev, torch.bfloat16, 224, 1000)
    loss = ops.softmax_cross_entropy(model(x), y)
    loss.backward()
    g = flat.groups["compute"].grad
    assert torch.isfinite(loss).item()
    assert torch.isfinite(g.float()).all().item() and g.float().abs().sum().item() > 0
