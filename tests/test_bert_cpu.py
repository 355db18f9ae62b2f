"""BERT reference path and transformer op mirrors on the CPU (the oracle of the fused GPU path)."""
import math

import torch
import torch.nn.functional as F

import dtg  # noqa: F401
from dtg.models.bert import BertConfig, BertForPreTraining, synthetic_batch
from dtg.ops import transformer as T


def test_dropout_mask_rate_and_determinism():
    k1 = T.dropout_keep(123, 200000, 0.1)
    k2 = T.dropout_keep(123, 200000, 0.1)
    k3 = T.dropout_keep(124, 200000, 0.1)
    assert torch.equal(k1, k2)
    assert not torch.equal(k1, k3)
    assert abs(k1.float().mean().item() - 0.9) < 0.005
    assert T.dropout_keep(5, 10, 0.0).all()


def test_dropout_hash_matches_scalar_definition():
    # fmix32(i * 0x9E3779B1 + seed) >= floor(p * 2^32), all arithmetic mod 2^32
    def fmix(h):
        h ^= h >> 16
        h = (h * 0x85EBCA6B) & 0xFFFFFFFF
        h ^= h >> 13
        h = (h * 0xC2B2AE35) & 0xFFFFFFFF
        return h ^ (h >> 16)
    seed, p = 0xDEADBEEF, 0.3
    th = int(p * 2 ** 32)
    keep = T.dropout_keep(seed, 1000, p)
    for i in range(0, 1000, 37):
        assert bool(keep[i]) == (fmix((i * 0x9E3779B1 + seed) & 0xFFFFFFFF) >= th)


def test_attention_dropout_pair_hash():
    """Attention-probability dropout: one fmix32 per pair of adjacent elements, low / high 16 bits against
    floor(p * 2^16) (the fused kernels hold 4 consecutive keys per lane: 2 hashes instead of 4)."""
    def fmix(h):
        h ^= h >> 16
        h = (h * 0x85EBCA6B) & 0xFFFFFFFF
        h ^= h >> 13
        h = (h * 0xC2B2AE35) & 0xFFFFFFFF
        return h ^ (h >> 16)
    seed, p = 0x1234567, 0.1
    th = int(p * 2 ** 16)
    keep = T.attn_dropout_keep(seed, 4000, p)
    for i in range(0, 4000, 29):
        h = fmix(((i >> 1) * 0x9E3779B1 + seed) & 0xFFFFFFFF)
        assert bool(keep[i]) == (((h >> 16) if i & 1 else (h & 0xFFFF)) >= th)
    big = T.attn_dropout_keep(99, 400000, 0.1).float()
    assert abs(big.mean().item() - 0.9) < 0.003
    # the two halves of a pair are (close to) independent draws
    ev, od = big[0::2], big[1::2]
    assert abs((ev * od).mean().item() - ev.mean().item() * od.mean().item()) < 0.003
    assert T.attn_dropout_keep(5, 10, 0.0).all()


def test_layer_norm_ref_matches_torch():
    x = torch.randn(10, 48)
    r = torch.randn(10, 48)
    g, b = torch.rand(48) + 0.5, torch.randn(48)
    y = T.layer_norm_ref(x, r, g, b, 1e-5)
    assert torch.allclose(y, F.layer_norm(x + r, (48,), g, b, 1e-5), atol=1e-5)


def test_attention_ref_matches_sdpa():
    B, S, nh, dh = 2, 16, 4, 8
    qkv = torch.randn(B * S, 3 * nh * dh)
    am = torch.ones(B, S)
    am[1, 10:] = 0
    out = T.attention_ref(qkv, T.mask_additive(am), B, S, nh)
    q, k, v = qkv.view(B, S, 3, nh, dh).permute(2, 0, 3, 1, 4)
    mask = (am > 0).view(B, 1, 1, S)
    ref = F.scaled_dot_product_attention(q, k, v, attn_mask=mask).permute(0, 2, 1, 3).reshape(B * S, -1)
    assert torch.allclose(out, ref, atol=1e-4)


def test_bert_reference_trains_and_is_deterministic():
    torch.manual_seed(0)
    cfg = BertConfig.tiny()
    m = BertForPreTraining(cfg)
    batch = synthetic_batch(4, 32, cfg, "cpu", max_predictions=5)
    opt = torch.optim.Adam(m.parameters(), lr=2e-3)
    losses = []
    for _ in range(25):
        loss = m(*batch)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(math.isfinite(v) for v in losses)
    assert losses[-1] < 0.6 * losses[0], losses
    # eval mode: no dropout, same output twice
    m.eval()
    with torch.no_grad():
        a, b = m(*batch), m(*batch)
    assert a.item() == b.item()


def test_bert_parameter_count_base():
    m = BertForPreTraining(BertConfig.base())
    n = sum(p.numel() for p in m.parameters())
    # BERT-base pre-training model: ~110M (+ padded-vocab rows and the MLM head)
    assert 109e6 < n < 112e6, n
