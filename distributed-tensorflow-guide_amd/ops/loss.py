"""Fused softmax cross-entropy (csrc/kernels/softmax_xent.hip).

The forward kernel computes the per-row loss and logsumexp; the backward kernel produces
d(loss)/d(logits) in one pass from the saved logits and lse, reading grad_output on the device (no
host sync and no separate rescale pass).  Rows whose label is < 0 are ignored (loss 0, gradient 0)
-- the BERT MLM head relies on this.
"""
import torch
import torch.nn.functional as F

from ._native import lib


class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, denom):
        logits, labels = logits.contiguous(), labels.contiguous()
        loss_rows, _, lse = lib().softmax_xent(logits, labels, 1.0 / denom, False)
        ctx.save_for_backward(logits, labels, lse)
        ctx.scale = 1.0 / denom
        return lib().row_sum(loss_rows, 1.0 / denom)  # one dtg reduction (fixed order), scaled

    @staticmethod
    def backward(ctx, g):
        logits, labels, lse = ctx.saved_tensors
        return lib().softmax_xent_bwd(logits, labels, lse, g, ctx.scale), None, None


def softmax_cross_entropy(logits, labels, num_valid=None):
    """Cross-entropy summed over rows with label >= 0 and divided by ``num_valid``
    (default: number of rows, i.e. the plain mean)."""
    labels = labels.long()
    denom = float(labels.numel() if num_valid is None else max(1, int(num_valid)))
    if logits.is_cuda:
        return _SoftmaxXent.apply(logits, labels, denom)
    mask = labels >= 0
    return F.cross_entropy(logits[mask].float(), labels[mask], reduction="sum") / denom
