"""BERT building blocks as single autograd nodes with hand-written backward passes (GPU, bf16).

Per encoder layer (T = batch*seq rows, H hidden, I intermediate; all GEMMs on the MFMA kernel):

  forward   qkv = x Wqkv^T + b                      (bias in the GEMM epilogue)
            ctx = attention(qkv)                     (2 strided-batched GEMMs + softmax/dropout kernel)
            x1  = LN(x + drop(ctx Wo^T + b))         (LN kernel fuses residual add + dropout)
            f1  = gelu(x1 W1^T + b1)                 (GELU in the epilogue; the same epilogue saves
                                                      GELU'(pre-activation) for backward, sharing its exp)
            out = LN(x1 + drop(f1 W2^T + b2))
  backward  LN kernels emit both the residual-path gradient and the dropout-masked branch gradient
            (masks regenerated from the counter hash); dgrad GEMMs accumulate the residual gradient
            (beta = 1) instead of a separate add; the saved GELU' is applied in the dgrad GEMM epilogue,
            which also column-sums the result into b1's gradient; the other bias gradients come from the
            LN backward or column-sum kernels into the fp32 flat grads;
            weight gradients accumulate straight into the flat gradient buffer (grad_sink).

The word embedding is tied to the MLM decoder: the MLM head adds its decoder gradient into the
embedding's flat gradient without notifying; the embedding node (which runs last in backward)
adds the lookup gradient and notifies once, so the all-reduce bucket holding the embedding sees
exactly one "ready" event per step.
"""

import torch

from ..ops._native import lib
from ..ops.gemm import gemm
from ..ops import transformer as T
from ..parallel import grad_sink, overlap


_ATTN = "fused"  # "fused" (attention.hip) or "gemm" (batched GEMMs + softmax; A/B tests)
# split-K workgroup target of the weight gradients when they run on the side stream (parallel/overlap.py); 0 = the
# GEMM's own default (512).  Module switch for the A/B tools (tools/bench_cfg.py DTG_AB_SET).
_WSPLIT_WGS = 0
# QKV bias gradient from the fused attention backward's epilogue (True) or a separate column-sum pass (A/B switch)
_FUSED_DBIAS = True
_wsplit_cache = {}


def _wgrad(dy, x, out):
    """out += dy^T x over the token dimension, with the side-stream split target."""
    tgt = _WSPLIT_WGS if overlap.enabled() else 0
    sk = 0
    if tgt > 0:
        key = (dy.shape[1], x.shape[1], dy.shape[0], tgt)
        sk = _wsplit_cache.get(key)
        if sk is None:
            sk = _wsplit_cache[key] = lib().gemm_pick_split(key[0], key[1], key[2], False, tgt)
    gemm(dy, False, x, False, out=out, beta=1.0, split_k=sk)


def _fused_attn(S, backward=True):
    return _ATTN == "fused" and lib().attn_fused_supported(S, 64, backward)


def _gacc(p):
    if grad_sink.enabled(p):
        return p.grad, True
    return torch.zeros_like(p, dtype=torch.float32 if p.dim() <= 1 else p.dtype), False


def _finish(params, accs, skip_notify=()):
    if not all(direct for _, direct in accs):
        # gradients without a flat buffer may have been written on the wgrad side stream: autograd can add
        # them into an existing .grad on the current stream as soon as we return them
        overlap.sync_current(accs[0][0].device)
    grads = []
    for p, (a, direct) in zip(params, accs):
        if direct:
            if not any(p is q for q in skip_notify):
                grad_sink.notify(p)
            grads.append(None)
        else:
            grads.append(a.to(p.dtype))
    return grads


class _LayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask_add, geom, holder, *params):
        L = lib()
        B, S, nh, eps, p_h, p_a, s_a, s_1, s_2 = geom
        w_qkv, b_qkv, w_o, b_o, g1, be1, w_1, b_1, w_2, b_2, g2, be2 = params
        qkv = gemm(x, True, w_qkv, True, bias=b_qkv)
        fused = _fused_attn(S) and w_qkv.shape[0] == 3 * nh * 64
        if fused:  # flash-style kernel: no [S, S] tensors; P recomputed in backward from the LSE
            cx, lse = L.attn_fused_fwd(qkv, mask_add, B, S, nh, p_a, s_a)
            P = Pd = lse
        else:
            cx, P, Pd = T.attention_fwd(qkv, mask_add, B, S, nh, p_a, s_a)
        ao = gemm(cx, True, w_o, True, bias=b_o)
        x1, s1, m1, r1 = L.ln_fwd(ao, x, g1, be1, eps, p_h, s_1, 0.0, 0, True)
        pre = torch.empty(x.shape[0], w_1.shape[0], device=x.device, dtype=x.dtype)
        f1 = torch.empty_like(pre)
        L.gemm(x1, True, w_1, True, f1, 1.0, 0.0, b_1, 2, 0, pre, 3)  # pre := gelu'(x1 W1^T + b1)
        f2 = gemm(f1, True, w_2, True, bias=b_2)
        out, s2, m2, r2 = L.ln_fwd(f2, x1, g2, be2, eps, p_h, s_2, 0.0, 0, True)
        ctx.geom = geom
        ctx.fused_attn = fused
        ctx.mask_add = mask_add
        ctx.mod_params = holder.params  # parameter objects: their .grad is the flat-buffer view
        ctx.save_for_backward(x, qkv, P, Pd, cx, x1, s1, m1, r1, pre, f1, s2, m2, r2, *params)
        return out

    @staticmethod
    def backward(ctx, dout):
        L = lib()
        B, S, nh, eps, p_h, p_a, s_a, s_1, s_2 = ctx.geom
        sv = ctx.saved_tensors
        x, qkv, P, Pd, cx, x1, s1, m1, r1, pre, f1, s2, m2, r2 = sv[:14]
        w_qkv, b_qkv, w_o, b_o, g1, be1, w_1, b_1, w_2, b_2, g2, be2 = sv[14:]
        mod_params = ctx.mod_params
        accs = [_gacc(p) for p in mod_params]
        (gw_qkv, _), (gb_qkv, _), (gw_o, _), (gb_o, _), (gg1, _), (gbe1, _), (gw_1, _), (gb_1, _), (gw_2, _), \
            (gb_2, _), (gg2, _), (gbe2, _) = accs
        H = x.shape[1]
        dout = dout.contiguous()
        # LN2: ds2 -> x1 (residual path), df2 -> f2 (dropout branch)
        ds2, df2 = L.ln_bwd(dout, s2, g2, m2, r2, gg2, gbe2, p_h, s_2, 0.0, 0, True, gb_2)  # + db2 = sum(df2)
        with overlap.wgrad_scope(df2, f1):  # weight gradients on the side stream (parallel/overlap.py)
            _wgrad(df2, f1, gw_2)                   # dW2 += df2^T f1
        dpre = torch.empty_like(pre)
        # df1 * gelu'(pre), and b1's gradient (column sums of it) in the same epilogue
        L.gemm(df2, True, w_2, False, dpre, 1.0, 0.0, None, 2, 0, pre, 4, colsum=gb_1)
        with overlap.wgrad_scope(dpre, x1):
            _wgrad(dpre, x1, gw_1)                  # dW1 += dpre^T x1
        if p_h <= 0:  # df2 aliases ds2: it has been consumed above; accumulate the residual grad into a copy
            ds2 = ds2.clone()
        gemm(dpre, True, w_1, False, out=ds2, beta=1.0)                       # dx1 = dpre W1 + ds2
        # LN1: ds1 -> x (residual), dao -> attention output projection
        ds1, dao = L.ln_bwd(ds2, s1, g1, m1, r1, gg1, gbe1, p_h, s_1, 0.0, 0, True, gb_o)  # + dbo = sum(dao)
        with overlap.wgrad_scope(dao, cx):
            _wgrad(dao, cx, gw_o)
        dcx = gemm(dao, True, w_o, False)
        if ctx.fused_attn and _FUSED_DBIAS and gb_qkv.dtype == torch.float32 and gb_qkv.is_contiguous():
            # the QKV bias gradient (column sums of dQKV) is added by the attention backward's epilogue
            dqkv = L.attn_fused_bwd(qkv, cx, dcx, P, ctx.mask_add, B, S, nh, p_a, s_a, gb_qkv)
        else:
            if ctx.fused_attn:
                dqkv = L.attn_fused_bwd(qkv, cx, dcx, P, ctx.mask_add, B, S, nh, p_a, s_a)
            else:
                dqkv = torch.empty_like(qkv)
                T.attention_bwd(dcx, qkv, P, Pd, B, S, nh, dqkv)
            L.colsum(dqkv, gb_qkv, True)
        with overlap.wgrad_scope(dqkv, x):
            _wgrad(dqkv, x, gw_qkv)
        if p_h <= 0:
            ds1 = ds1.clone()
        gemm(dqkv, True, w_qkv, False, out=ds1, beta=1.0)                     # dx = dqkv Wqkv + ds1
        grads = _finish(mod_params, accs)
        return (ds1, None, None, None, *grads)


class _Holder:
    """Carries the module's parameter objects into ctx (autograd only sees their tensors)."""
    __slots__ = ("params",)

    def __init__(self, params):
        self.params = params


def encoder_layer(layer, x, mask_add, B, S, cfg, p_h, p_a, s_a, s_1, s_2):
    params = layer.params()
    geom = (B, S, cfg.heads, cfg.eps, p_h, p_a, s_a, s_1, s_2)
    return _LayerFn.apply(x, mask_add, geom, _Holder(params), *params)


# ---- embeddings ----------------------------------------------------------------------------------------
class _EmbFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, tt, geom, holder, word, pos, typ, g, b):
        L = lib()
        S, eps, p, seed = geom
        s = L.emb_fwd(ids, tt, word, pos, typ, S)
        y, _, mean, rstd = L.ln_fwd(s, None, g, b, eps, 0.0, 0, p, seed, False)
        ctx.geom = geom
        ctx.mod_params = holder.params
        ctx.save_for_backward(ids, tt, s, mean, rstd, g)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = lib()
        S, eps, p, seed = ctx.geom
        ids, tt, s, mean, rstd, g = ctx.saved_tensors
        word, pos, typ, gam, bet = ctx.mod_params
        accs = [_gacc(q) for q in ctx.mod_params]
        (gw, _), (gp, _), (gt, _), (gg, _), (gb, _) = accs
        ds, _ = L.ln_bwd(dy.contiguous(), s, g, mean, rstd, gg, gb, 0.0, 0, p, seed, False)
        if not L.emb_word_bwd_owned(ds, ids, gw):  # sort-free, deterministic (heads.hip); wide H: sort
            srt, perm = torch.sort(ids)
            L.emb_word_bwd(ds, srt, perm, gw)
        L.emb_pos_bwd(ds, gp, S)
        if tt is not None:
            L.colsum(ds, gt.view(-1), True, tt, typ.shape[0])
        else:
            L.colsum(ds, gt[0], True)
        grads = _finish(ctx.mod_params, accs)
        return (None, None, None, None, *grads)


def embeddings(model, ids, tt, S, p, seed):
    e = model.emb
    cfg = model.cfg
    params = [e.word, e.pos, e.tok_type, e.ln_g, e.ln_b]
    ids1 = ids.reshape(-1).contiguous()
    tt1 = tt.reshape(-1).contiguous() if tt is not None else None
    return _EmbFn.apply(ids1, tt1, (S, cfg.eps, p, seed), _Holder(params), *params)


# ---- masked-LM head (transform + tied decoder + cross-entropy) -------------------------------------------
class _MLMFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hm, labels, geom, holder, w_t, b_t, g, b, word, dec_bias):
        L = lib()
        eps, denom = geom
        pre = torch.empty(hm.shape[0], w_t.shape[0], device=hm.device, dtype=hm.dtype)
        a = torch.empty_like(pre)
        L.gemm(hm, True, w_t, True, a, 1.0, 0.0, b_t, 2, 0, pre, 3)  # pre := gelu'(hm W^T + b), as in FFN1
        t, _, mean, rstd = L.ln_fwd(a, None, g, b, eps, 0.0, 0, 0.0, 0, False)
        logits = gemm(t, True, word, True, bias=dec_bias)
        loss_rows, _, lse = L.softmax_xent(logits, labels, 1.0 / denom, False)
        ctx.mod_params = holder.params
        ctx.scale = 1.0 / denom
        ctx.save_for_backward(hm, pre, a, mean, rstd, t, logits, labels, lse, w_t, g, word)
        return loss_rows.sum() / denom

    @staticmethod
    def backward(ctx, gout):
        L = lib()
        hm, pre, a, mean, rstd, t, logits, labels, lse, w_t, g, word = ctx.saved_tensors
        w_t_p, b_t_p, g_p, b_p, word_p, dec_p = ctx.mod_params
        accs = [_gacc(q) for q in ctx.mod_params]
        (gwt, _), (gbt, _), (gg, _), (gb, _), (gword, _), (gdec, _) = accs
        # d loss / d logits in one pass from the saved logits + lse, scaled by gout on the device
        dl = L.softmax_xent_bwd(logits, labels, lse, gout, ctx.scale)
        L.colsum(dl, gdec, True)
        gemm(dl, False, t, False, out=gword, beta=1.0)                 # tied decoder: dWemb += dl^T t
        dt = gemm(dl, True, word, False)                               # [P, H]
        da, _ = L.ln_bwd(dt, a, g, mean, rstd, gg, gb, 0.0, 0, 0.0, 0, False)
        dpre = L.mul_bf16(da, pre)                                     # pre holds gelu'(pre-activation)
        L.colsum(dpre, gbt, True)
        gemm(dpre, False, hm, False, out=gwt, beta=1.0)
        dhm = gemm(dpre, True, w_t, False)
        # the embedding node notifies the shared word-embedding gradient after adding its part
        grads = _finish(ctx.mod_params, accs, skip_notify=(word_p,))
        return (dhm, None, None, None, *grads)


def mlm_head(model, hm, labels, num_valid):
    params = [model.mlm_w, model.mlm_b, model.mlm_ln_g, model.mlm_ln_b, model.emb.word, model.mlm_bias]
    return _MLMFn.apply(hm.contiguous(), labels.contiguous(), (model.cfg.eps, float(num_valid)), _Holder(params),
                        *params)


# ---- both pre-training heads and the total loss as ONE node ----------------------------------------------
class _HeadsFn(torch.autograd.Function):
    """Masked-LM head (gather -> transform GEMM + GELU -> LN -> tied decoder GEMM -> softmax-xent) and the
    next-sentence head ([CLS] rows -> pooler GEMM with tanh epilogue -> 2-way softmax-xent) plus the sum of
    the two losses, all on dtg kernels (heads.hip, gemm.hip, softmax_xent.hip, transformer.hip): no
    index_select / slice / F.linear / F.cross_entropy on the step, and ``seq``'s gradient is assembled by
    a stream-ordered zero fill + two row scatters."""

    @staticmethod
    def forward(ctx, seq, pos, labels, nsp_labels, geom, holder, w_t, b_t, g, b, word, dec_bias, pool_w, pool_b,
                nsp_w, nsp_b):
        L = lib()
        eps, denom, B, S = geom
        H = seq.shape[1]
        hm = L.gather_rows(seq, pos, S)                                # masked rows, [B*P, H]
        pre = torch.empty(hm.shape[0], w_t.shape[0], device=hm.device, dtype=hm.dtype)
        a = torch.empty_like(pre)
        L.gemm(hm, True, w_t, True, a, 1.0, 0.0, b_t, 2, 0, pre, 3)  # pre := gelu'(hm W^T + b), as in FFN1
        t, _, mean, rstd = L.ln_fwd(a, None, g, b, eps, 0.0, 0, 0.0, 0, False)
        logits = gemm(t, True, word, True, bias=dec_bias)
        loss_rows, _, lse = L.softmax_xent(logits, labels, 1.0 / denom, False)
        mlm = L.row_sum(loss_rows, 1.0 / denom)
        cls = seq.view(B, S * H)[:, :H]                                # [CLS] rows, strided (no copy)
        pooled = gemm(cls, True, pool_w, True, bias=pool_b, act="tanh")
        total, probs = L.nsp_loss_fwd(pooled, nsp_w, nsp_b, nsp_labels, mlm)
        ctx.mod_params = holder.params
        ctx.scale = 1.0 / denom
        ctx.geom = geom
        ctx.save_for_backward(seq, pos, hm, pre, a, mean, rstd, t, logits, labels, lse, w_t, g, word, pooled, probs,
                              nsp_labels, pool_w, nsp_w)
        return total

    @staticmethod
    def backward(ctx, gout):
        L = lib()
        (seq, pos, hm, pre, a, mean, rstd, t, logits, labels, lse, w_t, g, word, pooled, probs, nsp_labels, pool_w,
         nsp_w) = ctx.saved_tensors
        _, _, B, S = ctx.geom
        H = seq.shape[1]
        params = ctx.mod_params
        word_p = params[4]
        accs = [_gacc(q) for q in params]
        (gwt, _), (gbt, _), (gg, _), (gb, _), (gword, _), (gdec, _), (gpw, _), (gpb, _), (gnw, _), (gnb, _) = accs
        gout = gout.float().reshape(1)
        # masked LM
        dl = L.softmax_xent_bwd(logits, labels, lse, gout, ctx.scale)
        L.colsum(dl, gdec, True)
        gemm(dl, False, t, False, out=gword, beta=1.0)                 # tied decoder: dWemb += dl^T t
        dt = gemm(dl, True, word, False)
        da, _ = L.ln_bwd(dt, a, g, mean, rstd, gg, gb, 0.0, 0, 0.0, 0, False)
        dpre = L.mul_bf16(da, pre)                                     # pre holds gelu'(pre-activation)
        L.colsum(dpre, gbt, True)
        gemm(dpre, False, hm, False, out=gwt, beta=1.0)
        dhm = gemm(dpre, True, w_t, False)
        # next sentence: dlogits -> (Wn, bn), tanh' -> pooler (Wp, bp) -> [CLS] rows
        dpp = L.nsp_loss_bwd(pooled, nsp_w, probs, nsp_labels, gout, gnw, gnb)
        L.colsum(dpp, gpb, True)
        cls = seq.view(B, S * H)[:, :H]
        gemm(dpp, False, cls, False, out=gpw, beta=1.0)
        dcls = gemm(dpp, True, pool_w, False)
        dseq = torch.empty_like(seq)
        L.zero_(dseq)
        L.scatter_rows_add(dseq, pos, dhm, S)
        L.scatter_rows_add(dseq, None, dcls, S)
        # the embedding node notifies the shared word-embedding gradient after adding its part
        grads = _finish(params, accs, skip_notify=(word_p,))
        return (dseq, None, None, None, None, None, *grads)


def heads_loss(model, seq, mlm_positions, mlm_labels, nsp_labels, num_valid, B, S):
    e = model.emb
    params = [model.mlm_w, model.mlm_b, model.mlm_ln_g, model.mlm_ln_b, e.word, model.mlm_bias, model.pool_w,
              model.pool_b, model.nsp_w, model.nsp_b]
    return _HeadsFn.apply(seq, mlm_positions.contiguous(), mlm_labels.reshape(-1).contiguous(), nsp_labels.contiguous(),
                          (model.cfg.eps, float(num_valid), B, S), _Holder(params), *params)
