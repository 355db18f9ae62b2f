"""MNIST CNN (BASELINE config 2) through the MirroredStrategy front end on the CPU (torch path)."""
import torch

import dtg  # noqa: F401
from dtg import ops
from dtg.models.mnist import MnistCNN, synthetic_mnist
from dtg.optim import FusedSGD
from dtg.parallel import MirroredStrategy


def test_mnist_cnn_learns_synthetic_digits():
    torch.manual_seed(0)
    s = MirroredStrategy("gloo", compute_dtype=torch.float32)
    assert s.num_replicas_in_sync == 1
    with s.scope():
        m = MnistCNN()
    tr = s.distribute(m, lambda f: FusedSGD(f, lr=0.01, momentum=0.9))
    losses = []
    for i in range(40):
        x, y = synthetic_mnist(64, "cpu", torch.float32, seed=i)
        losses.append(tr.step(lambda: ops.softmax_cross_entropy(m(x), y)).item())
    x, y = synthetic_mnist(256, "cpu", torch.float32, seed=999)
    with torch.no_grad():
        acc = (m(x).argmax(1) == y).float().mean().item()
    assert losses[-1] < losses[0]
    assert acc > 0.8, (acc, losses[::5])
