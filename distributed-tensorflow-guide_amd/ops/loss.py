"""Fused softmax cross-entropy (csrc/kernels/softmax_xent.hip).

The forward kernel also emits d(loss)/d(logits) for the requested mean, so backward is a rescale
by grad_output (a multiply by 1.0 in training).  Rows whose label is < 0 are ignored (loss 0,
gradient 0) -- the BERT MLM head relies on this.
"""
import torch
import torch.nn.functional as F

from ._native import lib


class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, denom):
        loss_rows, dlogits, _ = lib().softmax_xent(logits.contiguous(), labels.contiguous(), 1.0 / denom, True)
        ctx.save_for_backward(dlogits)
        return loss_rows.sum() / denom

    @staticmethod
    def backward(ctx, g):
        (dlogits,) = ctx.saved_tensors
        return dlogits * g.to(dlogits.dtype), None, None


def softmax_cross_entropy(logits, labels, num_valid=None):
    """Cross-entropy summed over rows with label >= 0 and divided by ``num_valid``
    (default: number of rows, i.e. the plain mean)."""
    labels = labels.long()
    denom = float(labels.numel() if num_valid is None else max(1, int(num_valid)))
    if logits.is_cuda:
        return _SoftmaxXent.apply(logits, labels, denom)
    mask = labels >= 0
    return F.cross_entropy(logits[mask].float(), labels[mask], reduction="sum") / denom
