"""Whole-step hipGraph capture (parallel/graphs.py): replaying the captured ResNet-50 / BERT training
step must train exactly like the eager step (same kernels, same order)."""
import pytest
import torch

import dtg  # noqa: F401
from dtg import ops
from dtg.models import resnet
from dtg.optim import FusedAdam, FusedSGD
from dtg.parallel import FlatParams, GraphedStep

pytestmark = pytest.mark.gpu


def _resnet_run(graphed, steps=6):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = resnet.resnet50(num_classes=10).to(dev).to(memory_format=torch.channels_last)
    flat = FlatParams(model)
    opt = FusedSGD(flat, lr=0.05, momentum=0.9, weight_decay=5e-5)
    x, y = resnet.synthetic_batch(8, dev, torch.bfloat16, 64, 10, seed=3)
    model.train()

    def step():
        loss = ops.softmax_cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        return loss

    fn = GraphedStep(step, warmup=2) if graphed else step
    losses = []
    n = 0
    while n < steps:
        loss = fn()
        # the capture call already ran `warmup` eager steps before its first replay
        n += (fn.warmup + 1) if (graphed and len(losses) == 0) else 1
        losses.append(float(loss.float().item()))
    torch.cuda.synchronize()
    return losses, flat.groups["compute"].master.clone(), flat.buffers.flat.clone()


def test_graphed_resnet_step_matches_eager():
    le, we, be = _resnet_run(False)
    lg, wg, bg = _resnet_run(True)
    assert all(map(lambda v: v == v, lg)), lg
    # BN statistics reduce with float atomics (order-dependent rounding): close, not bitwise
    assert abs(le[-1] - lg[-1]) <= 2e-2 * abs(le[-1]) + 1e-3, (le, lg)
    assert torch.allclose(we, wg, rtol=2e-2, atol=2e-3), (we - wg).abs().max()
    assert torch.allclose(be, bg, rtol=2e-2, atol=2e-3), (be - bg).abs().max()


def test_graph_replay_picks_up_new_inputs():
    """Static input buffers refilled in place between replays feed the next replay."""
    dev = torch.device("cuda")
    torch.manual_seed(0)
    from dtg.models.mnist import MnistCNN, synthetic_mnist
    model = MnistCNN().to(dev)
    flat = FlatParams(model)
    opt = FusedAdam(flat, lr=1e-3)
    x, y = synthetic_mnist(64, dev, torch.bfloat16, seed=0)
    xs, ys = x.clone(), y.clone()

    def step():
        loss = ops.softmax_cross_entropy(model(xs), ys)
        loss.backward()
        opt.step()
        return loss

    g = GraphedStep(step, warmup=1)
    g()
    hyper0 = float(opt.hyper[1].item())
    losses = []
    for i in range(20):
        xi, yi = synthetic_mnist(64, dev, torch.bfloat16, seed=i)
        xs.copy_(xi)
        ys.copy_(yi)
        losses.append(float(g().float().item()))
    # the device step counter (Adam bias correction) advances on every replay
    assert float(opt.hyper[1].item()) == hyper0 + 20
    assert losses[-1] < losses[0], losses
