"""Fused NHWC BatchNorm (+ residual add) (+ ReLU) backed by csrc/kernels/batchnorm.hip.

Activations are channels_last bf16, so a [N, C, H, W] tensor is an [N*H*W, C] row-major matrix
in memory and the kernels work on that view directly (no permute copies).
"""
import torch
import torch.nn.functional as F

from ._native import lib


def _as_rows(t):
    n, c, h, w = t.shape
    if not t.is_contiguous(memory_format=torch.channels_last):
        t = t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _from_rows(r, shape):
    n, c, h, w = shape
    return r.view(n, h, w, c).permute(0, 3, 1, 2)


class _BNActTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, weight, bias, running_mean, running_var, momentum, eps, relu):
        x2 = _as_rows(x)
        r2 = _as_rows(res) if res is not None else None
        y2, smean, sinv = lib().bn_fwd_train(x2, r2, weight, bias, running_mean, running_var, momentum, eps, relu)
        ctx.relu = relu
        ctx.has_res = res is not None
        ctx.shape = x.shape
        ctx.save_for_backward(x2, y2 if relu else None, weight, smean, sinv)
        return _from_rows(y2, x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, y2, weight, smean, sinv = ctx.saved_tensors
        dy2 = _as_rows(dy)
        dx2, dres2, dgamma, dbeta = lib().bn_bwd(dy2, y2, x2, weight, smean, sinv, ctx.relu, ctx.has_res)
        dx = _from_rows(dx2, ctx.shape)
        dres = _from_rows(dres2, ctx.shape) if ctx.has_res else None
        return dx, dres, dgamma, dbeta, None, None, None, None, None


def batch_norm_act(x, weight, bias, running_mean, running_var, training=True, momentum=0.1, eps=1e-5,
                   residual=None, relu=True):
    """y = relu?(BN(x) + residual?) for an NCHW tensor in channels_last memory."""
    if x.is_cuda and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0:
        if training:
            return _BNActTrain.apply(x, residual, weight, bias, running_mean, running_var, momentum, eps, relu)
        y2 = lib().bn_fwd_infer(_as_rows(x), _as_rows(residual) if residual is not None else None, weight, bias,
                                running_mean, running_var, eps, relu)
        return _from_rows(y2, x.shape)
    # reference path (CPU / odd shapes)
    y = F.batch_norm(x.float(), running_mean, running_var, weight, bias, training, momentum, eps).to(x.dtype)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y
