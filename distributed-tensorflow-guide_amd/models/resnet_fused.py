"""ResNet bottleneck as ONE autograd node with a hand-written backward (GPU, bf16, NHWC).

Everything runs on dtg's HIP kernels on [rows, channels] views of NHWC activations:

  forward   y1 = x W1^T (MFMA GEMM)        a1 = relu(bn1(y1))             (fused BN+ReLU)
            y2 = conv3x3(a1, W2, stride)  a2 = relu(bn2(y2))             (implicit-GEMM conv)
            y3 = a2 W3^T                  idn = x | bn_d(conv1x1_s(x, Wd))
            out = relu(bn3(y3) + idn)                                     (fused BN+add+ReLU)
  backward  the residual gradient that BN3's backward emits (dres) is the buffer the first
            conv's dgrad GEMM accumulates into (beta = 1): the "x is used twice" gradient sum
            costs no separate add kernel; conv weight gradients are accumulated straight into
            the flat gradient buffer and BN gamma/beta gradients are accumulated in the BN
            finalize kernel -- autograd sees no parameter gradients at all, the all-reduce
            buckets are notified through parallel/grad_sink.
Strided dgrads (3x3/s2 and the 1x1/s2 projection) run dtg's residue-class dgrad kernel; the
projection's accumulates (beta = 1) straight into the conv1 dgrad output.

BN statistics are fused into the producing GEMM/conv epilogue (csrc/include/dtg/bn_epi.cuh):
forward, every conv output's per-channel sum / sum of squares; backward, the dgrads feeding BN2 and
BN1 emit the relu-masked gradient plus sum(dp) and sum(dp*xhat).  Each BN then costs finalize +
one elementwise pass instead of a reduction pass + finalize + elementwise pass.  _FUSE = False
restores the separate statistics kernels (A/B tests).

BN3 of block i (relu(bn3(y3) + identity) = the block output = block i+1's input) is reduced one
block LATER: block i+1's last dgrad GEMM, the final writer of dL/d out_i, applies block i's relu
mask (out_i > 0, i.e. its own saved input) and reduces block i's BN3 statistics in its epilogue
(mode 3).  The two blocks meet through a _Bn3Link attached to the output tensor.  Block i uses the
partials only if the gradient it receives is that very buffer (so nothing else was summed into it
by autograd); otherwise it falls back to the full BN backward, which re-applies the (idempotent)
mask.
"""
import os

import torch
import torch.nn.functional as F

from ..ops import conv as conv_ops
from ..ops._native import lib
from ..ops.gemm import gemm
from ..parallel import grad_sink, overlap


def _rows(t):
    n, c, h, w = t.shape
    if not t.is_contiguous(memory_format=torch.channels_last):
        t = t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _mat(w):  # 1x1 conv weight [K, C, 1, 1] -> [K, C]
    return w.reshape(w.shape[0], w.shape[1]) if w.is_contiguous() else w.as_strided((w.shape[0], w.shape[1]),
                                                                                     (w.shape[1], 1))


def _krsc(w):  # channels_last [K, C, R, S] -> contiguous [K, R, S, C] view
    return w.permute(0, 2, 3, 1)


_FUSE = True  # BN statistics in the GEMM/conv epilogues (False: separate statistics kernels, for A/B tests)
_LINK = True  # cross-block BN3 reduction (needs _FUSE)
# linked stride-2 projection: its dgrad writes only the even (h, w) rows, which the next mode-3 GEMM alone
# reads (no zero-fill of a [N, H, W, C] gradient per stage transition); 0 restores the zero-filled form
_SUB2 = True
# (Round-3/4 experiments, removed in round 5 with their kernels -- git history has them: BN2 + relu applied in
# conv3's operand prologues instead of an apply pass, 14.46k vs 14.80k img/s at b512 (profiles/r03_bn2_prologue);
# BN3 / BN1 backward folded into the following 1x1 dgrads over [dp | y] along K, 14.2k vs 15.2k at b1024
# (profiles/r04_bn_fold).)
# _DXW = True: where the shape allows (stage 1: 256 x 64, bn_dx_wgrad_ok), conv3's weight gradient is computed inside
# BN3's dx pass on the main stream (csrc/kernels/bn_dx_wgrad.hip) instead of re-reading dx on the side stream:
# the backward is HBM-bound across both streams, and that re-read cost 0.3 ms of step per block
# (profiles/r04_dx_wgrad).
_DXW = True
_DXW2 = True  # ... and the stage-1 stride-1 projection's weight gradient in the dual form of that pass


class _Bn3Link:
    """Block i's BN3 tensors, filled with the mode-3 partials by block i+1's backward.  For a projection
    block also its shortcut BN's input and statistics (yd, md, idd): the same masked gradient feeds
    that BN, so block i+1's epilogue reduces its statistics too (part2)."""
    __slots__ = ("y3", "m3", "i3", "gamma", "beta", "bits", "yd", "md", "idd", "part", "part2", "dp")

    def __init__(self, y3, m3, i3, gamma, beta, bits, yd=None, md=None, idd=None):
        self.y3, self.m3, self.i3, self.gamma, self.beta = y3, m3, i3, gamma, beta
        self.bits = bits  # packed (out > 0): the relu mask, 1/16 of the bytes of re-reading out
        self.yd, self.md, self.idd = yd, md, idd
        self.part = self.part2 = self.dp = None


def _gacc(p):
    """The buffer a parameter's gradient is accumulated into (its flat view, or a fresh one)."""
    if grad_sink.enabled(p):
        return p.grad, True
    return torch.zeros_like(p, dtype=torch.float32 if p.dim() <= 1 else p.dtype), False


# _BITS = False: the backward recomputes BN1/BN2's relu masks from y and the BN statistics (mode 2)
# instead of reading the packed masks the forward apply wrote (mode 3, 1/16 of y's bytes)
_BITS = True


# Split-K targets (workgroups) of the weight gradients when they run on the side stream (parallel/overlap.py,
# one rank): there they overlap the dgrad / BN-backward chain, and fewer, longer splits (fewer fp32 partial
# slabs, fewer CUs taken from the main stream) measured faster -- ResNet-50 b512 13.99k -> 14.19k img/s
# for the 1x1 GEMM wgrads at 128 instead of 512, and +0.7 % for the 3x3 conv wgrads at 512 instead of
# 1024.  On the main stream (several ranks, or DTG_WGRAD_STREAM=0) the kernels' own defaults stay: there
# 128 ran 12.4k vs 13.67k img/s (profiles/r02_wgrad_split_policy).  DTG_RESNET_WSPLIT_WGS /
# DTG_RESNET_CWSPLIT_WGS override the side-stream targets (0: the defaults).  Round 4 at b1024, with the stage-1/2
# conv3 weight gradients fused into the dx passes: 1x1 at 256 beats 128 by 0.3-0.5 % (64: -6 %, 512: +0.1-0.4 %),
# and with the 1x1 at 256 the 3x3 at 256 beats 512 by 0.5 % (128: -3 %, 1024: -0.4 %; profiles/r04_wgrad_split).
_WSPLIT_WGS = int(os.environ.get("DTG_RESNET_WSPLIT_WGS", "256"))
_CWSPLIT_WGS = int(os.environ.get("DTG_RESNET_CWSPLIT_WGS", "256"))
_wsplit_cache = {}


def _wgrad(dy, x, out):
    """out (+)= dy^T x for [P, M] dy and [P, N] x (P pixels): a 1x1 conv weight gradient."""
    tgt = _WSPLIT_WGS if overlap.enabled() else 0
    key = (dy.shape[1], x.shape[1], dy.shape[0], tgt)
    sk = _wsplit_cache.get(key)
    if sk is None:
        sk = _wsplit_cache[key] = lib().gemm_pick_split(key[0], key[1], key[2], False, tgt) if tgt > 0 else 0
    gemm(dy, False, x, False, out=out, beta=1.0, split_k=sk)


def _conv_wgrad(dy4, x4, dw, st, pad):
    """dw (+)= 3x3 / strided conv weight gradient, with the side-stream split target (see above)."""
    lib().conv_wgrad(dy4, x4, dw, 1.0, st, pad, target_wgs=_CWSPLIT_WGS if overlap.enabled() else 0)


def _relu_bits(y):
    return torch.empty(y.shape[0], y.shape[1] // 8, device=y.device, dtype=torch.uint8) if _BITS else None


class _BottleneckFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, blk, link_in, holder, *params):
        L = lib()
        n, c, h, w = x.shape
        st = blk.c2.conv.stride
        width = blk.c1.conv.weight.shape[0]
        cout = blk.c3.conv.weight.shape[0]
        x2 = _rows(x)
        p_, q_ = (h + 2 - 3) // st + 1, (w + 2 - 3) // st + 1
        b1, b2, b3 = blk.c1.bn, blk.c2.bn, blk.c3.bn
        w1, w2, w3 = blk.c1.conv.weight, blk.c2.conv.weight, blk.c3.conv.weight
        if _FUSE:
            y1, p1 = L.gemm_bn(x2, _mat(w1), 1, pooled=True)
            bits1 = _relu_bits(y1)
            a1, m1, i1 = L.bn_fwd_part(y1, p1, None, b1.weight, b1.bias, b1.running_mean, b1.running_var,
                                       b1.momentum, b1.eps, True, bits=bits1)
            y2, p2 = L.conv_fwd_bn(a1.view(n, h, w, width), _krsc(w2), st, 1, pooled=True)
            y2 = y2.view(-1, width)
            bits2 = _relu_bits(y2)
            a2, m2, i2 = L.bn_fwd_part(y2, p2, None, b2.weight, b2.bias, b2.running_mean, b2.running_var,
                                       b2.momentum, b2.eps, True, bits=bits2)
            y3, p3 = L.gemm_bn(a2, _mat(w3), 1, pooled=True)
            ctx.bits12 = (bits1, bits2)
        else:
            y1 = gemm(x2, True, _mat(w1), True)
            a1, m1, i1 = L.bn_fwd_train(y1, None, b1.weight, b1.bias, b1.running_mean, b1.running_var, b1.momentum,
                                        b1.eps, True)
            y2 = L.conv_fwd(a1.view(n, h, w, width), _krsc(w2), st, 1).view(-1, width)
            a2, m2, i2 = L.bn_fwd_train(y2, None, b2.weight, b2.bias, b2.running_mean, b2.running_var, b2.momentum,
                                        b2.eps, True)
            y3 = gemm(a2, True, _mat(w3), True)
        yd = md = idd = None
        if blk.down is not None:
            bd, wd = blk.down.bn, blk.down.conv.weight
            if _FUSE:
                if st == 1:
                    yd, pd = L.gemm_bn(x2, _mat(wd), 1, pooled=True)
                else:
                    yd, pd = L.conv_fwd_bn(x2.view(n, h, w, c), _krsc(wd), st, 0, pooled=True)
                    yd = yd.view(-1, cout)
                idn = None  # applied together with BN3 below (no materialised identity branch)
            else:
                if st == 1:
                    yd = gemm(x2, True, _mat(wd), True)
                else:
                    yd = L.conv_fwd(x2.view(n, h, w, c), _krsc(wd), st, 0).view(-1, cout)
                idn, md, idd = L.bn_fwd_train(yd, None, bd.weight, bd.bias, bd.running_mean, bd.running_var,
                                              bd.momentum, bd.eps, False)
        else:
            idn = x2
        bits = None
        if _FUSE and _LINK:
            bits = torch.empty(y3.shape[0], cout // 8, device=y3.device, dtype=torch.uint8)
        if _FUSE and blk.down is not None:  # out = relu(bn3(y3) + bn_d(yd)) in one pass
            assert bd.momentum == b3.momentum and bd.eps == b3.eps
            out, m3, i3, md, idd = L.bn_fwd2_part(y3, p3, b3.weight, b3.bias, b3.running_mean, b3.running_var, yd, pd,
                                                  bd.weight, bd.bias, bd.running_mean, bd.running_var, b3.momentum,
                                                  b3.eps, bits=bits)
        elif _FUSE:
            out, m3, i3 = L.bn_fwd_part(y3, p3, idn, b3.weight, b3.bias, b3.running_mean, b3.running_var,
                                        b3.momentum, b3.eps, True, bits=bits)
        else:
            out, m3, i3 = L.bn_fwd_train(y3, idn, b3.weight, b3.bias, b3.running_mean, b3.running_var, b3.momentum,
                                         b3.eps, True)
        ctx.blk = blk
        ctx.link_in = link_in if (_FUSE and _LINK) else None
        ctx.link_out = _Bn3Link(y3, m3, i3, b3.weight, b3.bias, bits, yd, md, idd) if (_FUSE and _LINK) else None
        holder.append(ctx.link_out)
        ctx.geom = (n, c, h, w, st, width, cout, p_, q_)
        ctx.save_for_backward(x2, y1, a1, m1, i1, y2, a2, m2, i2, y3, out, m3, i3,
                              *((yd, md, idd) if yd is not None else ()))
        return out.view(n, p_, q_, cout).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dout):
        L = lib()
        blk = ctx.blk
        n, c, h, w, st, width, cout, p_, q_ = ctx.geom
        sv = ctx.saved_tensors
        x2, y1, a1, m1, i1, y2, a2, m2, i2, y3, out, m3, i3 = sv[:13]
        b1, b2, b3 = blk.c1.bn, blk.c2.bn, blk.c3.bn
        w1, w2, w3 = blk.c1.conv.weight, blk.c2.conv.weight, blk.c3.conv.weight
        params = [w1, b1.weight, b1.bias, w2, b2.weight, b2.bias, w3, b3.weight, b3.bias]
        if blk.down is not None:
            params += [blk.down.conv.weight, blk.down.bn.weight, blk.down.bn.bias]
        accs = [_gacc(p) for p in params]
        g = {id(p): a for p, (a, _) in zip(params, accs)}
        do = _rows(dout)
        # BN3 (+ residual, relu): dres is the gradient flowing into the identity branch
        lk = ctx.link_out
        dyd = None
        # conv3's weight gradient inside BN3's dx pass (_DXW)
        w3_kw = (dict(wact=a2, wgrad=g[id(w3)].view(cout, width))
                 if _DXW and a2 is not None and L.bn_dx_wgrad_ok(y3.shape[0], cout, width) else None)
        w3_done = wd_done = False
        if (lk is not None and lk.part is not None and do.data_ptr() == lk.dp.data_ptr()
                and do.shape == lk.dp.shape):
            # block i+1 already masked dL/d out (do is dp) and reduced this BN's statistics
            if lk.part2 is not None:  # ... and the shortcut BN's: both dx in one pass over dp
                bd = blk.down.bn
                kw = dict(w3_kw or {})
                if _DXW2 and w3_kw is not None and st == 1 and c == width == 64 and cout == 256:
                    # the stride-1 projection's weight gradient in the same pass (dyd^T x, stage 1)
                    kw.update(wact2=x2, wgrad2=g[id(blk.down.conv.weight)].view(cout, c))
                    wd_done = True
                dy3, dyd = L.bn_bwd2_part(do, y3, lk.part, b3.weight, m3, i3, g[id(b3.weight)], g[id(b3.bias)],
                                          sv[13], lk.part2, bd.weight, sv[14], sv[15], g[id(bd.weight)],
                                          g[id(bd.bias)], **kw)
                w3_done = w3_kw is not None
            else:
                dy3 = L.bn_bwd_part(do, y3, lk.part, b3.weight, m3, i3, False, g[id(b3.weight)], g[id(b3.bias)],
                                    **(w3_kw or {}))[0]
                w3_done = w3_kw is not None
            dres = do  # our own buffer (pointer-checked above): dx accumulates into it in place
        else:
            for pt in ((lk.part, lk.part2) if lk is not None else ()):
                if pt is not None:
                    pt.zero_()  # pooled slots must go back zeroed (see bn_part in csrc/bindings/ops.cc)
            dy3, dres, _, _ = L.bn_bwd(do, out, y3, b3.weight, m3, i3, True, True, g[id(b3.weight)],
                                       g[id(b3.bias)])
        if lk is not None:
            lk.part = lk.part2 = lk.dp = None
        # conv3 (1x1); with BN fusion its dgrad epilogue applies BN2's relu mask and reduces BN2's statistics
        bits1, bits2 = ctx.bits12 if _FUSE else (None, None)
        ctx.bits12 = None
        if _FUSE and bits2 is not None:  # relu mask from the forward's bits: mode 3 with nothing to accumulate
            dp2, q2 = L.gemm_bn(dy3, _mat(w3), 3, y2, m2, i2, b2.weight, b2.bias, mask=bits2, pooled=True)
        elif _FUSE:
            dp2, q2 = L.gemm_bn(dy3, _mat(w3), 2, y2, m2, i2, b2.weight, b2.bias, pooled=True)
        else:
            da2 = gemm(dy3, True, _mat(w3), False)
        if w3_done:
            pass  # accumulated by BN3's dx pass above
        else:
            with overlap.wgrad_scope(dy3, a2):
                _wgrad(dy3, a2, g[id(w3)].view(cout, width))
        # BN2 + conv2 (3x3)
        if _FUSE:
            dy2 = L.bn_bwd_part(dp2, y2, q2, b2.weight, m2, i2, False, g[id(b2.weight)], g[id(b2.bias)])[0]
        else:
            dy2 = L.bn_bwd(da2, a2, y2, b2.weight, m2, i2, True, False, g[id(b2.weight)], g[id(b2.bias)])[0]
        dy2_4 = dy2.view(n, p_, q_, width)
        if _FUSE:
            dp1, q1 = L.conv_dgrad_bn(dy2_4, _krsc(w2).contiguous(), h, w, st, 1, y1, m1, i1, b1.weight, b1.bias,
                                       pooled=True, bits=bits1)
            dp1 = dp1.view(-1, width)
        else:
            da1 = L.conv_dgrad(dy2_4, _krsc(w2).contiguous(), h, w, st, 1).view(-1, width)
        with overlap.wgrad_scope(dy2_4, a1):
            _conv_wgrad(dy2_4, a1.view(n, h, w, width), g[id(w2)].permute(0, 2, 3, 1), st, 1)
        # BN1 + conv1 (1x1): its dgrad accumulates into the identity-branch gradient
        dx_done = False
        sub2_hw = None
        lk_in = ctx.link_in
        ctx.link_in = None
        if lk_in is not None and lk_in.y3.shape != x2.shape:
            lk_in = None
        if _FUSE:
            dy1 = L.bn_bwd_part(dp1, y1, q1, b1.weight, m1, i1, False, g[id(b1.weight)], g[id(b1.bias)])[0]
        else:
            dy1 = L.bn_bwd(da1, a1, y1, b1.weight, m1, i1, True, False, g[id(b1.weight)], g[id(b1.bias)])[0]
        if blk.down is not None:
            yd, md, idd = sv[13:16]
            bd, wd = blk.down.bn, blk.down.conv.weight
            if dyd is None:
                dyd, _, _, _ = L.bn_bwd(dres, None, yd, bd.weight, md, idd, False, False, g[id(bd.weight)],
                                        g[id(bd.bias)])
            if st == 1:
                dx2 = gemm(dyd, True, _mat(wd), False)
                if not wd_done:
                    with overlap.wgrad_scope(dyd, x2):
                        _wgrad(dyd, x2, g[id(wd)].view(cout, c))
            elif lk_in is not None:  # projection dgrad first, so the conv1 dgrad GEMM is the last writer
                # only the even (h, w) rows of a stride-2 1x1 dgrad are written; the mode-3 GEMM below reads
                # just those (sub2_hw) instead of a zero-filled full tensor
                sub2 = st == 2 and _SUB2
                dx2 = L.conv_dgrad(dyd.view(n, p_, q_, cout), _krsc(wd).contiguous(), h, w, st, 0,
                                   zero_rest=not sub2).view(-1, c)
                if sub2:
                    sub2_hw = (h, w)
                with overlap.wgrad_scope(dyd, x2):
                    _conv_wgrad(dyd.view(n, p_, q_, cout), x2.view(n, h, w, c), g[id(wd)].permute(0, 2, 3, 1), st, 0)
            else:
                dx2 = gemm(dy1, True, _mat(w1), False)
                L.conv_dgrad(dyd.view(n, p_, q_, cout), _krsc(wd).contiguous(), h, w, st, 0, out=dx2.view(n, h, w, c),
                             beta=1.0)
                dx_done = True
                with overlap.wgrad_scope(dyd, x2):
                    _conv_wgrad(dyd.view(n, p_, q_, cout), x2.view(n, h, w, c), g[id(wd)].permute(0, 2, 3, 1), st, 0)
        else:
            dx2 = dres
        if not dx_done:
            if lk_in is not None:  # mode 3: finish the previous block's BN3 reduction in this epilogue
                part2 = None
                if lk_in.yd is not None:  # the previous block is a projection block: its shortcut BN too
                    part2 = L.bn_part_alloc(dp1, c, pooled=True)
                _, part = L.gemm_bn(dy1, _mat(w1), 3, lk_in.y3, lk_in.m3, lk_in.i3, lk_in.gamma, lk_in.beta,
                                    mask=lk_in.bits, out=dx2, pooled=True, x2=lk_in.yd, mean2=lk_in.md,
                                    invstd2=lk_in.idd, part2=part2, sub2_hw=sub2_hw)
                lk_in.part, lk_in.part2, lk_in.dp = part, part2, dx2
            else:
                gemm(dy1, True, _mat(w1), False, out=dx2, beta=1.0)
        with overlap.wgrad_scope(dy1, x2):
            _wgrad(dy1, x2, g[id(w1)].view(width, c))
        if not all(direct for _, direct in accs):
            overlap.sync_current(x2.device)  # side-stream wgrads land in these before autograd adds them
        grads = []
        for p, (a, direct) in zip(params, accs):
            if direct:
                grad_sink.notify(p)
                grads.append(None)
            else:
                grads.append(a.to(p.dtype))
        return (dx2.view(n, h, w, c).permute(0, 3, 1, 2), None, None, None, *grads)


def fused_ok(blk, x):
    ws = [blk.c1.conv.weight, blk.c2.conv.weight, blk.c3.conv.weight]
    return (blk.training and x.is_cuda and x.dtype == torch.bfloat16 and all(v.dtype == torch.bfloat16 for v in ws)
            and x.shape[1] % 64 == 0 and blk.c1.conv.weight.shape[0] % 64 == 0)


def bottleneck(blk, x):
    params = [blk.c1.conv.weight, blk.c1.bn.weight, blk.c1.bn.bias, blk.c2.conv.weight, blk.c2.bn.weight,
              blk.c2.bn.bias, blk.c3.conv.weight, blk.c3.bn.weight, blk.c3.bn.bias]
    if blk.down is not None:
        params += [blk.down.conv.weight, blk.down.bn.weight, blk.down.bn.bias]
    holder = []
    y = _BottleneckFn.apply(x, blk, getattr(x, "_dtg_bn3", None), holder, *params)
    if holder and holder[0] is not None:
        y._dtg_bn3 = holder[0]
    return y


# ---- stem: 7x7/2 conv (8-channel padded input) -> BN -> ReLU -> 3x3/2 max-pool, one autograd node ------
# csrc/kernels/stem.hip: the BN statistics come from the conv epilogue, BN+ReLU+pool is one pass over the
# conv output, and the backward recomputes the pre-pool gradient inside both BN-backward passes, so
# neither the BN output nor the pre-pool gradient (411 MB each at batch 256) is ever written.
# _STEM = False restores conv -> BN -> max-pool as separate ops (A/B tests).
_STEM = True
_POOL = (3, 2, 1)  # ResNet's stem max-pool: 3x3, stride 2, pad 1
# _STEM_YAM = True: the forward pool also saves y at each window's argmax ([N, 56, 56, 64], 1/4 of y), so the
# backward's BN statistics pass runs over the pooled tensors instead of gathering over y (csrc/kernels/stem.hip
# stem_bwd_pooled_stats_kernel; exact same terms, another summation order)
_STEM_YAM = True
# stem weight gradient (pixel-pair form): LDS schedule 3 (register-pipelined) and 512 split-K workgroups, measured
# 674 vs 748-878 us at b1024 for the default single stage / 1024 (tools/stem_wgrad_ab.py, profiles/r04_stem_pooled);
# 0 / 0 restore the defaults
_STEM_WG_SCHED = 3
_STEM_WG_WGS = 512


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, stem, w, gamma, beta):
        L = lib()
        n, c, h, wd = x.shape
        conv, bn = stem.conv, stem.bn
        k, _, r, s = w.shape
        st, pad = conv.stride, conv.padding
        if conv_ops.stem_pairs_ok(x, w, st):  # 4 channels x 2 pixels per 16-B chunk (ops/conv.py stem_pairs)
            x8, w8, (rk, sk) = conv_ops.stem_pairs(x, w, st, pad)
            y4, part = L.conv_fwd_c8(x8, w8, rk, sk, st, 0, True, stride_w=1)  # + BN statistics in the epilogue
            ctx.pairs = True
        else:
            ctx.pairs = False
            x8 = F.pad(x.permute(0, 2, 3, 1), (0, 8 - c)).contiguous()   # [N, H, W, 8]
            w8 = F.pad(w.permute(0, 2, 3, 1), (0, 8 - c)).reshape(k, r * s * 8)
            kp = (r * s * 8 + 63) // 64 * 64
            w8 = F.pad(w8, (0, kp - r * s * 8)).contiguous()           # [K, Kp], (r, s, c) columns
            y4, part = L.conv_fwd_c8(x8, w8, r, s, st, pad, True)      # + BN statistics in the epilogue
        yam_ok = _STEM_YAM and L.stem_pooled_stats_ok(y4.shape[-1])
        res = L.stem_bn_pool_fwd(y4, part, gamma, beta, bn.running_mean, bn.running_var, bn.momentum, bn.eps,
                                 *_POOL, save_yam=yam_ok)
        out, idx, smean, sinv = res[:4]
        ctx.save_for_backward(x8, y4, idx, smean, sinv, res[4] if yam_ok else None)
        ctx.stem = stem
        ctx.geom = (c, k, r, s, st, pad)
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dout):
        L = lib()
        x8, y4, idx, smean, sinv, yam = ctx.saved_tensors
        c, k, r, s, st, pad = ctx.geom
        stem = ctx.stem
        w, gamma, beta = stem.conv.weight, stem.bn.weight, stem.bn.bias
        (dg, dg_direct), (db, db_direct) = _gacc(gamma), _gacc(beta)
        do4 = dout.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
        dy4 = L.stem_bn_pool_bwd(do4, idx, y4, gamma, beta, smean, sinv, *_POOL, dgamma_acc=dg, dbeta_acc=db,
                                 yam=yam)[0]
        if ctx.pairs:  # pair form: the stored input is [N, Hp, Wp/2, 8]
            dwp = torch.empty(k, r, (s + 1) // 2, 8, device=x8.device, dtype=torch.float32)  # beta 0: overwritten
            L.conv_wgrad(dy4, x8, dwp, 0.0, st, 0, stride_w=1, sched=_STEM_WG_SCHED,
                         target_wgs=_STEM_WG_WGS)
        else:
            dwp = torch.empty(k, r, s, 8, device=x8.device, dtype=torch.float32)
            L.conv_wgrad(dy4, x8, dwp, 0.0, st, pad)
        grads = []
        if grad_sink.enabled(w):
            L.stem_dw_add(dwp, w.grad, ctx.pairs)  # straight into the flat gradient's [K, R, S, C] memory
            grad_sink.notify(w)
            grads.append(None)
        else:
            dw = conv_ops.stem_pairs_dw(dwp, c, s) if ctx.pairs else dwp[..., :c].permute(0, 3, 1, 2)
            grads.append(dw.to(w.dtype).contiguous(memory_format=torch.channels_last))
        for p, (a, direct) in ((gamma, (dg, dg_direct)), (beta, (db, db_direct))):
            if direct:
                grad_sink.notify(p)
                grads.append(None)
            else:
                grads.append(a.to(p.dtype))
        return (None, None, *grads)


def stem_ok(stem, x):
    w = stem.conv.weight
    return (_STEM and stem.training and x.is_cuda and x.dtype == torch.bfloat16 and not x.requires_grad
            and w.dtype == torch.bfloat16 and x.shape[1] <= 8 and w.shape[0] % 64 == 0
            and x.is_contiguous(memory_format=torch.channels_last))


def stem_pool(stem, x):
    """max_pool2d(relu(bn(conv(x))), 3, 2, 1) for the ResNet stem as one fused autograd node."""
    return _StemFn.apply(x, stem, stem.conv.weight, stem.bn.weight, stem.bn.bias)
