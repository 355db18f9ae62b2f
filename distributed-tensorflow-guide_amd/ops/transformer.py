"""Transformer ops on dtg's HIP kernels (csrc/kernels/transformer.hip) plus their PyTorch mirrors.

The mirrors define the semantics the kernels must reproduce (tests compare the two):

* ``dropout_keep``   -- the counter-hash dropout mask: element ``i`` of a tensor is kept iff
  ``fmix32(i * 0x9E3779B1 + seed) >= floor(p * 2**32)``.  The kernels regenerate it in backward,
  so no mask tensor is ever stored.
* ``attn_dropout_keep`` -- the attention-probability dropout: one hash per PAIR of adjacent elements, its
  low / high 16 bits against ``floor(p * 2**16)`` (the fused attention kernels hold 4 consecutive keys per lane).
* ``layer_norm_ref`` -- ``y = dropout_out(LN(res + dropout_in(h)))``.
* ``attention_ref``  -- softmax(QK^T/sqrt(d) + mask) -> attention dropout -> @V per head.

Not in the reference (TF1 toy models); this is the BERT-base slice of BASELINE.json
config 5.
"""
import math

import torch

from ._native import lib

_M32 = 0xFFFFFFFF


def _fmix32(h):
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _M32
    return h ^ (h >> 16)


def drop_threshold(p):
    if p <= 0:
        return 0
    return min(int(p * 4294967296.0), _M32)


def dropout_keep(seed, numel, p, device=None):
    """Boolean keep-mask of ``numel`` elements (flat index order), identical to the kernels'."""
    th = drop_threshold(p)
    if th == 0:
        return torch.ones(numel, dtype=torch.bool, device=device)
    idx = torch.arange(numel, dtype=torch.int64, device=device)
    h = _fmix32(((idx * 0x9E3779B1) + (seed & _M32)) & _M32)
    return h >= th


def attn_drop_threshold(p):
    """16-bit threshold of the attention-probability dropout (0 = off)."""
    if p <= 0:
        return 0
    t = int(p * 65536.0)
    return 0xFFFF if p * 65536.0 >= 65535.0 else max(t, 1)


def attn_dropout_keep(seed, numel, p, device=None):
    """Keep-mask of the attention-probability dropout, identical to attention.hip ``keep_attn`` and
    transformer.hip ``attn_softmax_fwd``: one hash per pair of adjacent elements, element ``i`` kept iff the
    low (even ``i``) / high (odd ``i``) 16 bits of ``fmix32((i >> 1) * 0x9E3779B1 + seed)`` are >= floor(p * 2**16)."""
    th = attn_drop_threshold(p)
    if th == 0:
        return torch.ones(numel, dtype=torch.bool, device=device)
    idx = torch.arange(numel, dtype=torch.int64, device=device)
    h = _fmix32((((idx >> 1) * 0x9E3779B1) + (seed & _M32)) & _M32)
    half = torch.where((idx & 1) == 1, h >> 16, h & 0xFFFF)
    return half >= th


def attn_dropout_ref(x, p, seed):
    if p <= 0:
        return x
    keep = attn_dropout_keep(seed, x.numel(), p, x.device).view(x.shape)
    return torch.where(keep, x / (1.0 - p), torch.zeros((), dtype=x.dtype, device=x.device))


def dropout_ref(x, p, seed):
    if p <= 0:
        return x
    keep = dropout_keep(seed, x.numel(), p, x.device).view(x.shape)
    return torch.where(keep, x / (1.0 - p), torch.zeros((), dtype=x.dtype, device=x.device))


def layer_norm_ref(h, res, gamma, beta, eps, p_in=0.0, seed_in=0, p_out=0.0, seed_out=0):
    s = dropout_ref(h, p_in, seed_in)
    if res is not None:
        s = s + res
    mean = s.mean(-1, keepdim=True)
    var = ((s - mean) ** 2).mean(-1, keepdim=True)
    y = (s - mean) * torch.rsqrt(var + eps) * gamma + beta
    return dropout_ref(y, p_out, seed_out)


def attention_ref(qkv, mask_add, B, S, nh, p=0.0, seed=0):
    """qkv [B*S, 3H] -> context [B*S, H] (the fused layer's attention, in plain torch)."""
    H = qkv.shape[1] // 3
    dh = H // nh
    q, k, v = qkv.view(B, S, 3, nh, dh).permute(2, 0, 3, 1, 4)  # [B, nh, S, dh] each
    sc = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
    if mask_add is not None:
        sc = sc + mask_add.view(B, 1, 1, S).to(sc.dtype)
    pr = torch.softmax(sc, dim=-1)
    pr = attn_dropout_ref(pr.reshape(-1, S), p, seed).view(B, nh, S, S)
    return (pr @ v).permute(0, 2, 1, 3).reshape(B * S, H)


def mask_additive(attention_mask):
    """[B, S] 1/0 attention mask -> fp32 additive key mask (0 / -10000, as in BERT)."""
    if attention_mask.is_cuda and attention_mask.dtype in (torch.int64, torch.float32):
        return lib().mask_additive(attention_mask.contiguous())  # one dtg kernel
    return (1.0 - attention_mask.float()) * -10000.0


# ---- thin wrappers over the native ops ------------------------------------------------------
def gemm_batched(a, a_kc, b, b_kc, c, M, N, K, lda, ldb, ldc, nb, nh, sa, sb, sc, alpha=1.0, beta=0.0):
    """Strided two-level batched GEMM; sa/sb/sc = (batch stride, head stride) in elements."""
    lib().gemm_strided_batched(a, a_kc, b, b_kc, c, M, N, K, lda, ldb, ldc, nb, nh, sa[0], sa[1], sb[0], sb[1],
                               sc[0], sc[1], alpha, beta)
    return c


def attention_fwd(qkv, mask_add, B, S, nh, p, seed):
    """Fused-path attention forward.  Returns (ctx [T,H], P, Pd)."""
    L = lib()
    T, H3 = qkv.shape
    H = H3 // 3
    dh = H // nh
    scores = torch.empty(B * nh * S, S, device=qkv.device, dtype=torch.float32)
    # scores[b,h] = Q_bh K_bh^T / sqrt(dh):   A = Q (KC, ld 3H)   B = K (KC, ld 3H)
    gemm_batched(qkv, True, qkv[:, H:], True, scores, S, S, dh, H3, H3, S, B, nh, (S * H3, dh), (S * H3, dh),
                 (nh * S * S, S * S), alpha=1.0 / math.sqrt(dh))
    P, Pd = L.attn_softmax_fwd(scores, mask_add, nh * S, p, seed)
    ctx = torch.empty(T, H, device=qkv.device, dtype=qkv.dtype)
    # ctx[b, :, h] = Pd_bh V_bh:   A = Pd (KC, ld S)   B = V (MC: [K=keys, N=dh], ld 3H)
    gemm_batched(Pd, True, qkv[:, 2 * H:], False, ctx, S, dh, S, S, H3, H, B, nh, (nh * S * S, S * S),
                 (S * H3, dh), (S * H, dh))
    return ctx, P, Pd


def attention_bwd(dctx, qkv, P, Pd, B, S, nh, dqkv):
    """Fused-path attention backward: fills dqkv [T, 3H] from dctx [T, H]."""
    L = lib()
    T, H3 = qkv.shape
    H = H3 // 3
    dh = H // nh
    dPd = torch.empty(B * nh * S, S, device=qkv.device, dtype=torch.float32)
    # dPd = dctx_bh V_bh^T:   A = dctx (KC, ld H)   B = V (KC, ld 3H)
    gemm_batched(dctx, True, qkv[:, 2 * H:], True, dPd, S, S, dh, H, H3, S, B, nh, (S * H, dh), (S * H3, dh),
                 (nh * S * S, S * S))
    # dV = Pd^T dctx:   A = Pd stored [q][k] -> MC (ld S)   B = dctx stored [q][d] -> MC (ld H)
    gemm_batched(Pd, False, dctx, False, dqkv[:, 2 * H:], S, dh, S, S, H, H3, B, nh, (nh * S * S, S * S),
                 (S * H, dh), (S * H3, dh))
    dS = L.attn_softmax_bwd(P, Pd, dPd, 1.0 / math.sqrt(dh))
    # dQ = dS K:   A = dS (KC, ld S)   B = K stored [k][d] -> MC (ld 3H)
    gemm_batched(dS, True, qkv[:, H:], False, dqkv, S, dh, S, S, H3, H3, B, nh, (nh * S * S, S * S), (S * H3, dh),
                 (S * H3, dh))
    # dK = dS^T Q:  A = dS stored [q][k] -> MC (ld S)   B = Q stored [q][d] -> MC (ld 3H)
    gemm_batched(dS, False, qkv, False, dqkv[:, H:], S, dh, S, S, H3, H3, B, nh, (nh * S * S, S * S), (S * H3, dh),
                 (S * H3, dh))
    return dqkv
