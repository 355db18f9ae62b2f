"""BERT (encoder + pre-training heads) in bf16 on dtg's kernels -- BASELINE.json config 5
("BERT-base bf16 sync DP on 8x MI355X (MFMA GEMM + embedding grad all-reduce)").

Not in the reference, which only trains a 2-parameter toy; this model is the
transformer workload of the north-star configs.  Architecture = Devlin et al. BERT: post-LN
encoder layers, tanh-GELU (as in the original TF code), dropout 0.1 on hidden states and attention
probabilities, MLM head tied to the word embedding, NSP head on the pooled [CLS] state.

Two forward paths with identical semantics:

* fused (GPU, bf16 weights): one autograd node per encoder layer / embedding / MLM head with a
  hand-written backward (models/bert_fused.py) -- MFMA GEMMs with fused bias/GELU epilogues,
  strided-batched attention GEMMs, LayerNorm kernels with fused residual + dropout, weight
  gradients accumulated straight into the flat gradient buffer;
* reference (any device/dtype): plain PyTorch with the same counter-hash dropout masks, used on
  the CPU and as the numerics oracle of the fused path.

The vocabulary is padded to a multiple of 64 (30522 -> 30528, as Megatron-style "padded vocab")
so every GEMM dimension is MFMA-tile friendly; padded ids never occur as inputs or labels.
"""
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import transformer as T
from . import bert_fused


@dataclass
class BertConfig:
    vocab_size: int = 30528
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    dropout: float = 0.1
    attn_dropout: float = 0.1
    eps: float = 1e-12
    init_std: float = 0.02

    @staticmethod
    def base():
        return BertConfig()

    @staticmethod
    def large():
        return BertConfig(hidden=1024, layers=24, heads=16, intermediate=4096)

    @staticmethod
    def tiny():
        return BertConfig(vocab_size=512, hidden=64, layers=2, heads=2, intermediate=256, max_position=64)


def _normal(shape, std):
    return nn.Parameter(torch.randn(*shape) * std)


def _zeros(n):
    return nn.Parameter(torch.zeros(n))


def _ones(n):
    return nn.Parameter(torch.ones(n))


class BertEmbeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        H = cfg.hidden
        self.word = _normal((cfg.vocab_size, H), cfg.init_std)
        self.pos = _normal((cfg.max_position, H), cfg.init_std)
        self.tok_type = _normal((cfg.type_vocab, H), cfg.init_std)
        self.ln_g = _ones(H)
        self.ln_b = _zeros(H)


class BertLayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        H, I = cfg.hidden, cfg.intermediate
        s = cfg.init_std
        self.w_qkv = _normal((3 * H, H), s)  # [Wq; Wk; Wv] as one [3H, H] GEMM operand
        self.b_qkv = _zeros(3 * H)
        self.w_o = _normal((H, H), s)
        self.b_o = _zeros(H)
        self.ln1_g = _ones(H)
        self.ln1_b = _zeros(H)
        self.w_1 = _normal((I, H), s)
        self.b_1 = _zeros(I)
        self.w_2 = _normal((H, I), s)
        self.b_2 = _zeros(H)
        self.ln2_g = _ones(H)
        self.ln2_b = _zeros(H)

    def params(self):
        return [self.w_qkv, self.b_qkv, self.w_o, self.b_o, self.ln1_g, self.ln1_b, self.w_1, self.b_1, self.w_2,
                self.b_2, self.ln2_g, self.ln2_b]


class BertForPreTraining(nn.Module):
    def __init__(self, cfg=None, seed=1234):
        super().__init__()
        self.cfg = cfg = cfg or BertConfig.base()
        H = cfg.hidden
        self.emb = BertEmbeddings(cfg)
        self.layers = nn.ModuleList([BertLayer(cfg) for _ in range(cfg.layers)])
        s = cfg.init_std
        self.pool_w = _normal((H, H), s)
        self.pool_b = _zeros(H)
        self.mlm_w = _normal((H, H), s)
        self.mlm_b = _zeros(H)
        self.mlm_ln_g = _ones(H)
        self.mlm_ln_b = _zeros(H)
        self.mlm_bias = _zeros(cfg.vocab_size)
        self.nsp_w = _normal((2, H), s)
        self.nsp_b = _zeros(2)
        self.fused = True
        self.fused_heads = True  # MLM + NSP heads + losses as one node on dtg kernels (bert_fused.heads_loss)
        self.seed = seed
        self._step = 0

    # -- dropout seeds: one per (step, layer, site); regenerated (not stored) in backward --------------
    def _seed(self, layer, site):
        return (self.seed * 0x9E3779B1 + self._step * 0x85EBCA6B + layer * 0x27D4EB2F + site * 0x165667B1) & 0xFFFFFFFF

    def fused_ok(self, ids):
        H, S = self.cfg.hidden, ids.shape[1]
        w2 = [p for p in self.parameters() if p.dim() == 2]
        w1 = [p for p in self.parameters() if p.dim() == 1]
        return (self.fused and ids.is_cuda and all(p.dtype == torch.bfloat16 for p in w2)
                and all(p.dtype == torch.float32 for p in w1) and H % 64 == 0 and (H // self.cfg.heads) % 8 == 0
                and S % 8 == 0 and self.cfg.type_vocab <= 2 and self.cfg.vocab_size % 8 == 0)

    def forward(self, ids, token_types, attention_mask, mlm_positions, mlm_labels, nsp_labels, num_valid=None):
        """Pre-training loss = masked-LM cross-entropy (mean over ``num_valid`` predictions,
        default: all ``mlm_positions``) + next-sentence cross-entropy (mean over the batch).

        ids/token_types/attention_mask: [B, S]; mlm_positions/mlm_labels: [B, P] (label -1 = no
        prediction); nsp_labels: [B]."""
        if self.training:
            self._step += 1
        B, S = ids.shape
        cfg = self.cfg
        p_h = cfg.dropout if self.training else 0.0
        p_a = cfg.attn_dropout if self.training else 0.0
        mask_add = T.mask_additive(attention_mask) if attention_mask is not None else None
        labels = mlm_labels.reshape(-1)
        nv = labels.numel() if num_valid is None else num_valid
        if self.fused_ok(ids):
            seq = bert_fused.embeddings(self, ids, token_types, S, p_h, self._seed(0, 0))
            for i, layer in enumerate(self.layers):
                seq = bert_fused.encoder_layer(layer, seq, mask_add, B, S, cfg, p_h, p_a, self._seed(i + 1, 1),
                                               self._seed(i + 1, 2), self._seed(i + 1, 3))
            if self.fused_heads and mlm_positions.dtype == torch.long and nsp_labels.dtype == torch.long:
                return bert_fused.heads_loss(self, seq, mlm_positions, mlm_labels, nsp_labels, nv, B, S)
            mlm = bert_fused.mlm_head(self, seq.index_select(0, self._flat_pos(mlm_positions, S)), labels, nv)
        else:
            seq = self._reference_encoder(ids, token_types, mask_add, p_h, p_a)
            mlm = self._reference_mlm(seq.index_select(0, self._flat_pos(mlm_positions, S)), labels, nv)
        cls = seq.view(B, S, -1)[:, 0]
        pooled = torch.tanh(F.linear(cls, self.pool_w, self.pool_b.to(cls.dtype)))
        nsp_logits = F.linear(pooled, self.nsp_w, self.nsp_b.to(pooled.dtype))
        nsp = F.cross_entropy(nsp_logits.float(), nsp_labels)
        return mlm + nsp

    @staticmethod
    def _flat_pos(mlm_positions, S):
        B = mlm_positions.shape[0]
        return (mlm_positions + torch.arange(B, device=mlm_positions.device).unsqueeze(1) * S).reshape(-1)

    # -- plain PyTorch path (CPU, and the oracle of the fused path) -------------------------------------------
    def _reference_encoder(self, ids, token_types, mask_add, p_h, p_a):
        cfg = self.cfg
        B, S = ids.shape
        e = self.emb
        x = e.word[ids] + e.pos[:S].unsqueeze(0)
        if token_types is not None:
            x = x + e.tok_type[token_types]
        x = T.layer_norm_ref(x.reshape(B * S, -1), None, e.ln_g.to(x.dtype), e.ln_b.to(x.dtype), cfg.eps,
                             p_out=p_h, seed_out=self._seed(0, 0))
        for i, L in enumerate(self.layers):
            dt = x.dtype
            qkv = F.linear(x, L.w_qkv, L.b_qkv.to(dt))
            ctx = T.attention_ref(qkv, mask_add, B, S, cfg.heads, p_a, self._seed(i + 1, 1))
            ao = F.linear(ctx, L.w_o, L.b_o.to(dt))
            x1 = T.layer_norm_ref(ao, x, L.ln1_g.to(dt), L.ln1_b.to(dt), cfg.eps, p_in=p_h, seed_in=self._seed(i + 1, 2))
            f1 = F.gelu(F.linear(x1, L.w_1, L.b_1.to(dt)), approximate="tanh")
            f2 = F.linear(f1, L.w_2, L.b_2.to(dt))
            x = T.layer_norm_ref(f2, x1, L.ln2_g.to(dt), L.ln2_b.to(dt), cfg.eps, p_in=p_h, seed_in=self._seed(i + 1, 3))
        return x

    def _reference_mlm(self, hm, labels, num_valid):
        dt = hm.dtype
        t = F.gelu(F.linear(hm, self.mlm_w, self.mlm_b.to(dt)), approximate="tanh")
        t = T.layer_norm_ref(t, None, self.mlm_ln_g.to(dt), self.mlm_ln_b.to(dt), self.cfg.eps)
        logits = F.linear(t, self.emb.word, self.mlm_bias.to(dt)).float()
        valid = labels >= 0
        return F.cross_entropy(logits[valid], labels[valid], reduction="sum") / num_valid


def synthetic_batch(batch, seq_len, cfg, device, max_predictions=20, seed=0, real_vocab=30522):
    """Random pre-training batch of BERT's input signature (no dataset: synthetic, see bench.py)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    V = min(real_vocab, cfg.vocab_size)
    ids = torch.randint(0, V, (batch, seq_len), generator=g)
    tt = (torch.arange(seq_len).unsqueeze(0) >= seq_len // 2).long().expand(batch, seq_len).contiguous()
    am = torch.ones(batch, seq_len, dtype=torch.long)
    P = min(max_predictions, seq_len - 1)
    pos = torch.stack([torch.randperm(seq_len - 1, generator=g)[:P] + 1 for _ in range(batch)])
    lab = torch.randint(0, V, (batch, P), generator=g)
    nsp = torch.randint(0, 2, (batch,), generator=g)
    return tuple(t.to(device) for t in (ids, tt, am, pos, lab, nsp))
