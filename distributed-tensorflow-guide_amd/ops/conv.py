"""2-D convolution on NHWC (channels_last) bf16 activations.

Dispatch (set ``DTG_CONV_IMPL=miopen`` to force the library path for A/B runs):
  * 1x1 / stride 1 / pad 0  -> the MFMA GEMM (csrc/kernels/gemm.hip) on the [N*H*W, C] row view:
        fwd  Y  = X  W^T      dgrad dX = dY W      wgrad dW = dY^T X
  * k x k implicit-GEMM     -> csrc/kernels/conv.hip when built with it (see ``_IMPLICIT``)
  * everything else         -> MIOpen through torch (stem 7x7/Cin=3 etc.)
"""
import os

import torch
import torch.nn.functional as F

from ..parallel import grad_sink
from .gemm import gemm

_IMPL = os.environ.get("DTG_CONV_IMPL", "dtg")


def _rows(t):
    n, c, h, w = t.shape
    if not t.is_contiguous(memory_format=torch.channels_last):
        t = t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


class _Conv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        n, c, h, wd = x.shape
        cout = w.shape[0]
        x2 = _rows(x)
        w2 = w.as_strided((cout, c), (c, 1)) if w.is_contiguous(memory_format=torch.channels_last) or w.is_contiguous() \
            else w.reshape(cout, c).contiguous()
        y2 = gemm(x2, True, w2, True)
        ctx.save_for_backward(x2, w2)
        ctx.shape = (n, c, h, wd)
        ctx.wshape = w.shape
        ctx.param = w if grad_sink.enabled(w) else None
        return y2.view(n, h, wd, cout).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x2, w2 = ctx.saved_tensors
        n, c, h, wd = ctx.shape
        dy2 = _rows(dy)
        dx2 = gemm(dy2, True, w2, False) if ctx.needs_input_grad[0] else None
        dx = dx2.view(n, h, wd, c).permute(0, 3, 1, 2) if dx2 is not None else None
        p = ctx.param
        if p is not None:
            # wgrad accumulates straight into the flat gradient buffer (beta = 1)
            gemm(dy2, False, x2, False, out=p.grad.view(w2.shape), beta=1.0)
            grad_sink.notify(p)
            return dx, None
        dw2 = gemm(dy2, False, x2, False)
        return dx, dw2.view(ctx.wshape)


def conv2d(x, w, stride=1, padding=0):
    kh, kw = w.shape[2], w.shape[3]
    if (_IMPL == "dtg" and x.is_cuda and x.dtype == torch.bfloat16 and kh == 1 and kw == 1 and stride == 1
            and padding == 0 and x.shape[1] % 8 == 0 and w.shape[0] % 8 == 0):
        return _Conv1x1.apply(x, w)
    return F.conv2d(x, w, None, stride, padding)
