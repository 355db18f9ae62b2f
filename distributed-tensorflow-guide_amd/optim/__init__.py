"""Optimizers: fused flat-buffer applies (north-star models)."""
from .fused import FusedSGD, FusedAdam, FusedAdagrad, make_optimizer  # noqa: F401
