"""Loader for the native HIP kernel module ``dtg._C``.

GPU tensors always go through the hand-written gfx950 kernels; if the extension is missing on a
machine that has a GPU we raise instead of silently falling back (build with
``python tools/build_ext.py``).  CPU tensors (used by the gloo/CPU plumbing tests and the
parameter-server toy examples) take the PyTorch reference path in each op.
"""
import importlib

_C = None
_ERR = None


def lib():
    global _C, _ERR
    if _C is None:
        try:
            _C = importlib.import_module("dtg._C")
        except ImportError as e:  # pragma: no cover - depends on build state
            _ERR = e
            raise RuntimeError(
                "dtg native kernels (dtg._C) are not built or failed to load: %r. "
                "Run `python tools/build_ext.py` (gfx950)." % (e,)) from e
    return _C


def available():
    try:
        lib()
        return True
    except RuntimeError:
        return False


_LAB = None


def lab():
    """The A/B lab extension ``dtg._lab`` (csrc/lab: kernels that are NOT part of the production ``_C`` --
    negative results and main-loop candidates; build with ``python tools/build_ext.py --only lab``).  Its
    kernels reuse production symbols of ``_C`` (e.g. the split-K reduction), so ``_C`` is first made global
    (``RTLD_NOLOAD | RTLD_GLOBAL`` on the already-loaded library) before ``_lab`` is imported."""
    global _LAB
    if _LAB is None:
        import ctypes
        import os
        c = lib()
        ctypes.CDLL(c.__file__, mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL | os.RTLD_NOW)
        _LAB = importlib.import_module("dtg._lab")
    return _LAB
