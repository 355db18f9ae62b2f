"""Utilities for the GPU training path (SURVEY §5.1 tracing / §5.5 metrics).

* :func:`trace_range` / :func:`traced` -- roctx ranges (``torch.cuda.nvtx`` is roctx on ROCm) around
  forward, backward, each all-reduce bucket, the optimizer apply and the async-PS push / pull.
  Visible in ``rocprofv3 --marker-trace``; off unless ``DTG_TRACE=1`` (no cost on the hot path).
* :class:`StepTimer` -- per-step GPU time from HIP events recorded on the compute stream, read back
  lazily (no synchronisation inside the training loop); examples/sec from the batch size.
* :class:`MetricsLogger` -- JSONL metrics records (one JSON object per line), rank-tagged.

The session-level equivalents for the TF-style API are ``train.hooks.StepCounterHook`` and
``train.hooks.ProfilerHook``.
"""
from .trace import trace_enabled, trace_range, traced  # noqa: F401
from .timing import StepTimer  # noqa: F401
from .metrics import MetricsLogger  # noqa: F401
