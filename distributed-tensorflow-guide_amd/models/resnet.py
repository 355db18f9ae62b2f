"""ResNet-50 (v1.5: stride on the 3x3 conv) in NHWC bf16 -- the BASELINE north-star model
("ResNet-50 bf16 sync all-reduce DP on 8x MI355X").  Not in the reference (which trains a
2-parameter toy); built for the BASELINE.json configs 3 and 4.

Every BatchNorm is fused with its ReLU, and the last BN of each bottleneck also with the
residual add (one HIP kernel pass instead of three).
"""
import torch
import torch.nn as nn

from . import resnet_fused
from ..ops.pool import max_pool2d, global_avg_pool
from .layers import ConvBN, Linear


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1):
        super().__init__()
        cout = width * self.expansion
        self.c1 = ConvBN(cin, width, 1)
        self.c2 = ConvBN(width, width, 3, stride, 1)
        self.c3 = ConvBN(width, cout, 1, zero_init=True)
        self.down = ConvBN(cin, cout, 1, stride) if (stride != 1 or cin != cout) else None

    fused = True  # one autograd node with a hand-written backward on GPU (resnet_fused.py)

    def forward(self, x):
        if self.fused and resnet_fused.fused_ok(self, x):
            return resnet_fused.bottleneck(self, x)
        idn = self.down(x, relu=False) if self.down is not None else x
        y = self.c1(x)
        y = self.c2(y)
        return self.c3(y, residual=idn, relu=True)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, width=64):
        super().__init__()
        self.stem = ConvBN(3, width, 7, 2, 3)
        blocks = []
        cin = width
        for i, n in enumerate(layers):
            w = width * (2 ** i)
            for j in range(n):
                blocks.append(Bottleneck(cin, w, stride=2 if (j == 0 and i > 0) else 1))
                cin = w * Bottleneck.expansion
        self.blocks = nn.Sequential(*blocks)
        self.fc = Linear(cin, num_classes, init_std=0.01)

    def forward(self, x):
        if resnet_fused.stem_ok(self.stem, x):  # conv + BN + ReLU + max-pool as one node (stem.hip)
            x = resnet_fused.stem_pool(self.stem, x)
        else:
            x = self.stem(x)
            x = max_pool2d(x, 3, 2, 1)
        x = self.blocks(x)
        x = global_avg_pool(x)
        return self.fc(x)


def resnet50(num_classes=1000):
    return ResNet((3, 4, 6, 3), num_classes)


def resnet18_like_tiny(num_classes=10):
    """Small variant for CPU tests (same code paths, 1 block per stage, narrow)."""
    return ResNet((1, 1, 1, 1), num_classes, width=8)


def synthetic_batch(batch, device, dtype=torch.bfloat16, image=224, num_classes=1000, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(batch, 3, image, image, generator=g).to(device=device, dtype=dtype)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, num_classes, (batch,), generator=g).to(device)
    return x, y
