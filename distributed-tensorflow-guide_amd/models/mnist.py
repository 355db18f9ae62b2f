"""MNIST CNN (BASELINE.json config 2: "MNIST CNN sync all-reduce bf16 on 1 MI355X (single-replica
MirroredStrategy-equiv)").  The classic TF tutorial network: conv5x5(1->32)+ReLU, max-pool 2,
conv5x5(32->64)+ReLU, max-pool 2, FC 3136->1024 + ReLU, FC 1024->10.

On the GPU every op is a dtg kernel: the small-channel convs run as im2col + MFMA GEMM with the
bias/ReLU epilogue (ops.conv.conv2d_bias_act), pooling on the NHWC max-pool kernel, the FCs on the
MFMA GEMM, the loss on the fused softmax-xent kernel.  Not in the reference (it trains a toy
2-parameter model); there is no dataset offline, so ``synthetic_mnist`` draws a
learnable synthetic task of the same shape (10 random prototype digits + noise).
"""
import math

import torch
import torch.nn as nn

from ..ops.conv import conv2d_bias_act
from ..ops.pool import max_pool2d
from .layers import Linear


class MnistCNN(nn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.w1 = nn.Parameter(torch.randn(32, 1, 5, 5) * math.sqrt(2.0 / 25))
        self.b1 = nn.Parameter(torch.zeros(32))
        self.w2 = nn.Parameter(torch.randn(64, 32, 5, 5) * math.sqrt(2.0 / 800))
        self.b2 = nn.Parameter(torch.zeros(64))
        self.fc1 = Linear(7 * 7 * 64, 1024, act="relu")
        self.fc2 = Linear(1024, num_classes)

    def forward(self, x):
        dt = x.dtype
        x = conv2d_bias_act(x, self.w1.to(dt), self.b1, 1, 2, "relu")
        x = max_pool2d(x, 2, 2)
        x = conv2d_bias_act(x, self.w2.to(dt), self.b2, 1, 2, "relu")
        x = max_pool2d(x, 2, 2)
        x = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)  # NHWC flatten (a view for channels_last)
        return self.fc2(self.fc1(x))


def synthetic_mnist(n, device, dtype=torch.bfloat16, seed=0, noise=0.5):
    """(images [n,1,28,28], labels [n]): label-dependent prototypes + Gaussian noise."""
    g = torch.Generator(device="cpu").manual_seed(1234)
    protos = torch.rand(10, 1, 28, 28, generator=g)
    g2 = torch.Generator(device="cpu").manual_seed(seed)
    y = torch.randint(0, 10, (n,), generator=g2)
    x = (protos[y] - 0.5) * 2.0 + noise * torch.randn(n, 1, 28, 28, generator=g2)
    return x.to(device=device, dtype=dtype).contiguous(memory_format=torch.channels_last), y.to(device)
