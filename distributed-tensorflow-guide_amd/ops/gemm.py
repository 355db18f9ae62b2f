"""Dense layers on the hand-written MFMA GEMM (csrc/kernels/gemm.hip).

All three training GEMMs run without transposes: the kernel reads each operand either
K-contiguous (ds_read_b128) or MN-contiguous (ds_read_b64_tr_b16 hardware transpose).

    forward   Y  = X  W^T + b     A = X  [M,K] (KC)   B = W [N,K] (KC)
    dgrad     dX = dY W           A = dY [M,N] (KC)   B = W [N,K] (MC: reduction over N rows)
    wgrad     dW = dY^T X         A = dY [M,N] (MC)   B = X [M,K] (MC)
"""
import torch
import torch.nn.functional as F

from ._native import lib
from ..parallel import grad_sink

ACT = {None: 0, "none": 0, "relu": 1, "gelu": 2, "tanh": 3}


def gemm(a, a_kc, b, b_kc, out=None, alpha=1.0, beta=0.0, bias=None, act=None, split_k=0, out_dtype=None):
    """out[M,N] = act(alpha * op(a) @ op(b) + beta * out + bias) on MFMA.

    a_kc: ``a`` is stored [M,K] (else [K,M]);  b_kc: ``b`` is stored [N,K] (else [K,N]).
    """
    M = a.shape[0] if a_kc else a.shape[1]
    N = b.shape[0] if b_kc else b.shape[1]
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=out_dtype or a.dtype)
    lib().gemm(a, a_kc, b, b_kc, out, alpha, beta, bias, ACT[act], split_k)
    return out


def _gemm_ok(x2, w):
    return (x2.is_cuda and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x2.shape[1] % 8 == 0
            and w.shape[0] % 8 == 0 and x2.shape[0] % 8 == 0)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, w, b, act):
        bias32 = b.float() if b is not None and b.dtype != torch.float32 else b
        pre = None
        if act == "gelu":
            # keep the pre-activation for the GELU derivative
            pre = gemm(x2, True, w, True, bias=bias32)
            y = gelu_fwd(pre)
        else:
            y = gemm(x2, True, w, True, bias=bias32, act=act)
        ctx.act = act
        ctx.has_bias = b is not None
        ctx.bias_param = b if grad_sink.enabled(b) else None
        ctx.bias_dtype = b.dtype if b is not None else None
        ctx.param = w if grad_sink.enabled(w) else None
        ctx.save_for_backward(x2, w, pre if act == "gelu" else (y if act == "relu" else None))
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, w, saved = ctx.saved_tensors
        dy = dy.contiguous()
        if ctx.act == "gelu":
            dy = gelu_bwd(dy, saved)
        elif ctx.act == "relu":
            dy = dy * (saved > 0)
        dx = gemm(dy, True, w, False) if ctx.needs_input_grad[0] else None  # [M,K]
        db = None
        if ctx.bias_param is not None and dy.shape[1] % 8 == 0:
            lib().colsum(dy, ctx.bias_param.grad, True, None, 1)  # bias gradient straight into the flat buffer
            grad_sink.notify(ctx.bias_param)
        elif ctx.has_bias:
            db = dy.float().sum(0).to(ctx.bias_dtype)
        p = ctx.param
        if p is not None:
            gemm(dy, False, x2, False, out=p.grad, beta=1.0)  # wgrad straight into the flat buffer
            grad_sink.notify(p)
            return dx, None, db, None
        dw = gemm(dy, False, x2, False, out_dtype=w.dtype)  # [N,K]
        return dx, dw, db, None


def linear(x, weight, bias=None, act=None):
    """y = act(x @ weight^T + bias).  GPU bf16 -> MFMA kernel, otherwise torch."""
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    if _gemm_ok(x2, weight):
        y = _Linear.apply(x2.contiguous(), weight, bias, act)
    else:
        y = F.linear(x2, weight, bias.to(x2.dtype) if bias is not None else None)
        if act == "relu":
            y = F.relu(y)
        elif act == "gelu":
            y = F.gelu(y, approximate="tanh")
    return y.reshape(*shp[:-1], weight.shape[0])


def gelu_fwd(x):
    return F.gelu(x, approximate="tanh")


def gelu_bwd(dy, x):
    xf = x.float()
    k = 0.7978845608028654
    u = k * (xf + 0.044715 * xf ** 3)
    t = torch.tanh(u)
    d = 0.5 * (1 + t) + 0.5 * xf * (1 - t * t) * k * (1 + 3 * 0.044715 * xf * xf)
    return (dy.float() * d).to(dy.dtype)
