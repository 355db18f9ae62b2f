"""Building blocks that route compute through dtg.ops (HIP kernels on GPU).

Conventions: activations are NCHW-shaped tensors in channels_last memory (NHWC), compute dtype
bf16; conv/linear weights are bf16 views of the flat master buffer once wrapped by
:class:`dtg.parallel.FlatParams` (they are cast on the fly before that); norm parameters and
running statistics stay fp32.
"""
import math

import torch
import torch.nn as nn

from .. import ops


def _cast(w, dtype):
    return w if w.dtype == dtype else w.to(dtype)


class Conv2d(nn.Module):
    def __init__(self, cin, cout, k, stride=1, padding=0):
        super().__init__()
        self.stride, self.padding, self.k = stride, padding, k
        w = torch.empty(cout, cin, k, k)
        nn.init.kaiming_normal_(w, mode="fan_out", nonlinearity="relu")
        self.weight = nn.Parameter(w.contiguous(memory_format=torch.channels_last))

    def forward(self, x):
        return ops.conv2d(x, _cast(self.weight, x.dtype), self.stride, self.padding)


class BatchNorm2d(nn.Module):
    """BatchNorm with the following residual add and ReLU fused into the same kernel pass."""

    def __init__(self, c, momentum=0.1, eps=1e-5, zero_init=False):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(c) if zero_init else torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.momentum, self.eps = momentum, eps

    def forward(self, x, residual=None, relu=True):
        return ops.batch_norm_act(x, self.weight, self.bias, self.running_mean, self.running_var, self.training,
                                  self.momentum, self.eps, residual, relu)


class ConvBN(nn.Module):
    def __init__(self, cin, cout, k, stride=1, padding=0, zero_init=False):
        super().__init__()
        self.conv = Conv2d(cin, cout, k, stride, padding)
        self.bn = BatchNorm2d(cout, zero_init=zero_init)

    def forward(self, x, residual=None, relu=True):
        return self.bn(self.conv(x), residual, relu)


class Linear(nn.Module):
    def __init__(self, cin, cout, bias=True, act=None, init_std=None):
        super().__init__()
        w = torch.empty(cout, cin)
        if init_std is None:
            nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        else:
            nn.init.normal_(w, std=init_std)
        self.weight = nn.Parameter(w)
        self.bias = nn.Parameter(torch.zeros(cout)) if bias else None
        self.act = act

    def forward(self, x):
        return ops.linear(x, _cast(self.weight, x.dtype), self.bias, self.act)
