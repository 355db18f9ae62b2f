"""2-D convolution on NHWC (channels_last) bf16 activations -- dtg's own MFMA kernels.

Dispatch (module attribute ``_IMPL = "miopen"`` forces the library path for A/B runs):
  * 1x1 / stride 1 / pad 0 -> the MFMA GEMM (csrc/kernels/gemm.hip) on the [N*H*W, C] row view:
        fwd  Y  = X  W^T      dgrad dX = dY W      wgrad dW = dY^T X
  * k x k, C % 64 == 0, K % 64 == 0 -> implicit-GEMM conv (csrc/kernels/conv.hip):
        fwd, dgrad and wgrad at any stride (strided dgrad: one dense launch per residue class of dx)
  * small channel counts (C % 64 != 0, K % 8 == 0: MNIST's 1/32-channel convs) -> im2col kernel +
    MFMA GEMM with the bias/ReLU epilogue; dgrad = GEMM + col2im gather kernel
    (``conv2d_bias_act``)
  * <= 8 input channels with K % 64 == 0 (the 7x7/2 Cin=3 stem) -> implicit-GEMM conv on the input
    zero-padded to 8 channels (one pixel = one 16-B chunk, csrc/kernels/conv.hip ``conv_fwd_c8``) and
    the same kernel's wgrad; no dgrad (the stem's input is the image).  With <= 4 channels and stride 2
    the input is instead packed as pixel PAIRS (``stem_pairs``): 4 channels x 2 adjacent pixels per
    16-B chunk, so the 7x7 filter's K dimension is 7 x 4 x 8 = 224 (padded to 256) instead of
    7 x 7 x 8 = 392 (padded to 448) -- 43 % fewer MFMA operations and half the input bytes
  * everything else -> MIOpen through torch
Weight gradients are accumulated straight into the flat gradient buffer (see parallel/grad_sink).
"""

import torch
import torch.nn.functional as F

from ..parallel import grad_sink
from ._native import lib
from .gemm import gemm

_IMPL = "dtg"
_PAIRS = True  # the pixel-pair stem conv (stem_pairs); False: the 8-channel padded form


def _rows(t):
    n, c, h, w = t.shape
    if not t.is_contiguous(memory_format=torch.channels_last):
        t = t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _nhwc(t):
    if not t.is_contiguous(memory_format=torch.channels_last):
        t = t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 2, 3, 1)


class _Conv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        n, c, h, wd = x.shape
        cout = w.shape[0]
        x2 = _rows(x)
        w2 = w.as_strided((cout, c), (c, 1)) if (w.is_contiguous(memory_format=torch.channels_last)
                                                  or w.is_contiguous()) else w.reshape(cout, c).contiguous()
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


class _ConvImplicit(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad):
        x4 = _nhwc(x)
        w4 = _nhwc(w)  # [K, R, S, C]
        y4 = lib().conv_fwd(x4.contiguous(), w4.contiguous(), stride, pad)
        ctx.save_for_backward(x4, w4)
        ctx.stride, ctx.pad = stride, pad
        ctx.xshape, ctx.w = x.shape, w
        ctx.param = w if grad_sink.enabled(w) else None
        return y4.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x4, w4 = ctx.saved_tensors
        st, pad = ctx.stride, ctx.pad
        dy4 = _nhwc(dy).contiguous()
        n, c, h, wd = ctx.xshape
        k, r, s = w4.shape[0], w4.shape[1], w4.shape[2]
        dx = None
        if ctx.needs_input_grad[0]:
            if lib().conv_supported(c, k, r, s, st, pad, 1):
                dx = lib().conv_dgrad(dy4, w4.contiguous(), h, wd, st, pad).permute(0, 3, 1, 2)
            else:  # unsupported channel counts: MIOpen
                w_cl = w4.permute(0, 3, 1, 2)
                dx = torch.nn.grad.conv2d_input(ctx.xshape, w_cl, dy4.permute(0, 3, 1, 2), st, pad)
        p = ctx.param
        if p is not None:
            lib().conv_wgrad(dy4, x4.contiguous(), p.grad.permute(0, 2, 3, 1), 1.0, st, pad)
            grad_sink.notify(p)
            return dx, None, None, None
        dw4 = torch.empty_like(w4.contiguous())
        lib().conv_wgrad(dy4, x4.contiguous(), dw4, 0.0, st, pad)
        return dx, dw4.permute(0, 3, 1, 2), None, None


def stem_pairs(x, w, stride, pad):
    """Pixel-pair form of a stride-2 conv over <= 4 input channels (the ResNet stem).

    Input column iw = 2q - pad + s of output column q lands, in a copy of x padded by `pad` on every side
    and to 4 channels, at padded column 2q + s: the 16-B pair chunk u = q + s // 2, half s % 2.  So the
    conv is a (stride 2, stride_w 1, pad 0) conv over [N, Hp, Wp/2, 8] "pixels" (two real pixels x 4
    channels each) with an R x ceil(S/2) filter whose 8 channels are (s % 2, c).

    Returns (xp [N, Hp, Wp/2, 8], wp [K, ceil64(R*S2*8)], (R, S2)) for conv_fwd_c8/conv_wgrad with
    stride=stride, pad=0, stride_w=1.  x: NCHW-shaped (channels_last preferred), w: [K, C, R, S].
    """
    n, c, h, wd = x.shape
    k, _, r, s = w.shape
    s2 = (s + 1) // 2
    q = (wd + 2 * pad - s) // stride + 1
    wp = max(wd + 2 * pad, 2 * (q - 1) + 2 * s2)
    wp += wp & 1
    if x.is_cuda and x.dtype == torch.bfloat16:  # one packing pass (csrc/kernels/stem.hip)
        xp = lib().stem_pack_pairs(_nhwc(x).contiguous(), pad, wp)
    else:
        xp = F.pad(_nhwc(x), (0, 4 - c, pad, wp - wd - pad, pad, pad)).contiguous()   # [N, Hp, Wp, 4]
        xp = xp.view(n, h + 2 * pad, wp // 2, 8)
    if (w.is_cuda and w.dtype == torch.bfloat16 and w.is_contiguous(memory_format=torch.channels_last)
            and c <= 4):  # one dtg packing pass (csrc/kernels/stem.hip)
        return xp, lib().stem_pack_weights(w), (r, s2)
    w4 = F.pad(w.permute(0, 2, 3, 1), (0, 4 - c, 0, 2 * s2 - s)).reshape(k, r * s2 * 8)  # (r, s//2, s%2, c)
    kp = (r * s2 * 8 + 63) // 64 * 64
    return xp, F.pad(w4, (0, kp - r * s2 * 8)).contiguous(), (r, s2)


def stem_pairs_ok(x, w, stride):
    return x.shape[1] <= 4 and stride == 2 and _PAIRS


def stem_pairs_dw(dwp, c, s):
    """[K, R, S2, 8] pair-form weight gradient -> [K, C, R, S] (a view)."""
    k, r, s2, _ = dwp.shape
    return dwp.view(k, r, s2 * 2, 4)[:, :, :s, :c].permute(0, 3, 1, 2)


class _ConvC8(torch.autograd.Function):
    """Few-channel input conv (ResNet stem): input padded to 8 channels, weights to [K, ceil64(R*S*8)]."""

    @staticmethod
    def forward(ctx, x, w, stride, pad):
        n, c, h, wd = x.shape
        k, _, r, s = w.shape
        if stem_pairs_ok(x, w, stride):
            x8, w8, (rk, sk) = stem_pairs(x, w, stride, pad)
            y4, _ = lib().conv_fwd_c8(x8, w8, rk, sk, stride, 0, stride_w=1)
            ctx.geom = (c, k, r, s, stride, pad, True)
        else:
            x8 = F.pad(_nhwc(x), (0, 8 - c)).contiguous()          # [N, H, W, 8]
            w8 = F.pad(w.permute(0, 2, 3, 1), (0, 8 - c)).reshape(k, r * s * 8)
            kp = (r * s * 8 + 63) // 64 * 64
            w8 = F.pad(w8, (0, kp - r * s * 8)).contiguous()       # [K, Kp], (r, s, c) columns
            y4, _ = lib().conv_fwd_c8(x8, w8, r, s, stride, pad)
            ctx.geom = (c, k, r, s, stride, pad, False)
        ctx.save_for_backward(x8)
        ctx.param = w if grad_sink.enabled(w) else None
        ctx.needs_dx = ctx.needs_input_grad[0]
        return y4.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        (x8,) = ctx.saved_tensors
        c, k, r, s, st, pad, pairs = ctx.geom
        if ctx.needs_dx:
            raise NotImplementedError("input gradient of the 8-channel stem conv (the image needs none)")
        if pairs:
            dwp = torch.zeros(k, r, (s + 1) // 2, 8, device=x8.device, dtype=torch.float32)
            lib().conv_wgrad(_nhwc(dy).contiguous(), x8, dwp, 0.0, st, 0, stride_w=1)
            dw = stem_pairs_dw(dwp, c, s)
        else:
            dw8 = torch.zeros(k, r, s, 8, device=x8.device, dtype=torch.float32)
            lib().conv_wgrad(_nhwc(dy).contiguous(), x8, dw8, 0.0, st, pad)
            dw = dw8[..., :c].permute(0, 3, 1, 2)                    # [K, C, R, S] view
        p = ctx.param
        if p is not None:
            p.grad.add_(dw.to(p.grad.dtype))
            grad_sink.notify(p)
            return None, None, None, None
        return None, dw.to(ctx.saved_tensors[0].dtype).contiguous(memory_format=torch.channels_last), None, None


def _kp(w):
    return (w.shape[1] * w.shape[2] * w.shape[3] + 7) // 8 * 8


def _w_cols(w, kp):
    """[K, C, R, S] -> [K, Kp] in (r, s, c) column order, zero padded."""
    k = w.shape[0]
    w2 = w.permute(0, 2, 3, 1).reshape(k, -1)
    if w2.shape[1] != kp:
        w2 = torch.nn.functional.pad(w2, (0, kp - w2.shape[1]))
    return w2.contiguous()


class _ConvIm2col(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, act):
        n, c, h, wd = x.shape
        k, _, r, s = w.shape
        kp = _kp(w)
        cols = lib().im2col(_nhwc(x).contiguous(), r, s, stride, pad, kp)
        w2 = _w_cols(w, kp)
        bias32 = b.float() if b is not None else None
        y2 = gemm(cols, True, w2, True, bias=bias32, act=act)
        p_, q_ = (h + 2 * pad - r) // stride + 1, (wd + 2 * pad - s) // stride + 1
        ctx.save_for_backward(cols, w2, y2 if act == "relu" else None)
        ctx.geom = (n, c, h, wd, k, r, s, stride, pad, p_, q_, kp)
        ctx.act = act
        ctx.has_bias = b is not None
        ctx.bdtype = b.dtype if b is not None else None
        ctx.wdtype = w.dtype
        return y2.view(n, p_, q_, k).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        cols, w2, y2 = ctx.saved_tensors
        n, c, h, wd, k, r, s, stride, pad, p_, q_, kp = ctx.geom
        dy2 = _rows(dy)
        if ctx.act == "relu":
            dy2 = dy2 * (y2 > 0)
        dw2 = gemm(dy2, False, cols, False, out_dtype=torch.float32)  # [K, Kp]
        dw = dw2[:, :r * s * c].reshape(k, r, s, c).permute(0, 3, 1, 2).to(ctx.wdtype)
        db = dy2.float().sum(0).to(ctx.bdtype) if ctx.has_bias else None
        dx = None
        if ctx.needs_input_grad[0]:
            dcols = gemm(dy2, True, w2, False)  # [NPQ, Kp]
            dx = lib().col2im(dcols, n, h, wd, c, r, s, stride, pad).permute(0, 3, 1, 2)
        return dx, dw, db, None, None, None


def conv2d_bias_act(x, w, bias=None, stride=1, padding=0, act=None):
    """act(conv2d(x, w) + bias) for any channel count: im2col + MFMA GEMM (GPU bf16), torch otherwise."""
    if x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.shape[0] % 8 == 0:
        return _ConvIm2col.apply(x.contiguous(memory_format=torch.channels_last), w, bias, stride, padding, act)
    y = F.conv2d(x, w, bias.to(x.dtype) if bias is not None else None, stride, padding)
    return F.relu(y) if act == "relu" else y


def conv2d(x, w, stride=1, padding=0):
    kh, kw = w.shape[2], w.shape[3]
    cin, cout = x.shape[1], w.shape[0]
    if _IMPL == "dtg" and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16:
        if kh == 1 and kw == 1 and stride == 1 and padding == 0 and cin % 8 == 0 and cout % 8 == 0:
            return _Conv1x1.apply(x, w)
        if cin % 64 == 0 and cout % 64 == 0:
            return _ConvImplicit.apply(x, w, stride, padding)
        if cin <= 8 and cout % 64 == 0 and not x.requires_grad:
            return _ConvC8.apply(x, w, stride, padding)
    return F.conv2d(x, w, None, stride, padding)
