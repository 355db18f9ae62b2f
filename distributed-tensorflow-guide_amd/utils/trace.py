"""roctx ranges for the training path.

``torch.cuda.nvtx.range_push/pop`` call roctx on ROCm builds of PyTorch, so these ranges show up in
``rocprofv3 --marker-trace`` next to the kernel trace: which kernels ran inside forward, backward,
a given all-reduce bucket, the fused apply, an async-PS push or pull.  Disabled unless
``DTG_TRACE=1`` (or :func:`set_trace`): then a range is one branch on a module global.
"""
import contextlib
import functools
import os

_ON = os.environ.get("DTG_TRACE", "0") == "1"
_nvtx = None


def trace_enabled():
    return _ON


def set_trace(on):
    global _ON
    _ON = bool(on)


def _backend():
    global _nvtx
    if _nvtx is None:
        try:
            import torch
            _nvtx = torch.cuda.nvtx if torch.cuda.is_available() else False
        except Exception:  # no GPU build: ranges are no-ops
            _nvtx = False
    return _nvtx


@contextlib.contextmanager
def trace_range(name):
    """``with trace_range("dtg.backward"): ...`` -- a roctx range when tracing is on."""
    nv = _backend() if _ON else False
    if not nv:
        yield
        return
    nv.range_push(name)
    try:
        yield
    finally:
        nv.range_pop()


def traced(name):
    """Decorator form of :func:`trace_range`."""
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **kw):
            if not _ON:
                return fn(*a, **kw)
            with trace_range(name):
                return fn(*a, **kw)
        return wrapper
    return deco
