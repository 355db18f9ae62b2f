"""NHWC pooling on dtg's HIP kernels (csrc/kernels/pool.hip).

Tensors are NCHW-shaped views of channels_last storage (as everywhere in dtg's conv nets).  The
max-pool saves a uint8 window index per output element; its backward is a gather (no atomics).
CPU / other layouts fall back to torch.
"""
import torch
import torch.nn.functional as F

from ._native import lib


def _nhwc(x):
    return x.permute(0, 2, 3, 1)  # channels_last NCHW view -> contiguous NHWC view


def _ok(x):
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last))


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, pad):
        y, idx = lib().maxpool_fwd(_nhwc(x), k, s, pad)
        ctx.geom = (x.shape[2], x.shape[3], k, s, pad)
        ctx.save_for_backward(idx)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        H, W, k, s, pad = ctx.geom
        dyn = _nhwc(dy.contiguous(memory_format=torch.channels_last))
        dx = lib().maxpool_bwd(dyn, idx, H, W, k, s, pad)
        return dx.permute(0, 3, 1, 2), None, None, None


class _GlobalAvg(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return lib().avgpool_fwd(_nhwc(x))

    @staticmethod
    def backward(ctx, dy):
        H, W = ctx.hw
        return lib().avgpool_bwd(dy.contiguous(), H, W).permute(0, 3, 1, 2)


def max_pool2d(x, kernel_size, stride=None, padding=0):
    stride = stride or kernel_size
    if _ok(x):
        return _MaxPool.apply(x, kernel_size, stride, padding)
    return F.max_pool2d(x, kernel_size, stride, padding)


def global_avg_pool(x):
    """[N, C, H, W] -> [N, C] mean over H, W."""
    if _ok(x):
        return _GlobalAvg.apply(x)
    return x.mean(dim=(2, 3))
