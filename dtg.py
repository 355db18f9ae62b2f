"""Import shim: exposes the ``distributed-tensorflow-guide_amd/`` package as ``dtg``.

The package directory name contains hyphens (it mirrors the reference repository's name), which
Python cannot import directly.  Importing this module loads that directory as the package ``dtg``
and replaces itself in ``sys.modules`` so that ``import dtg.models`` etc. work normally.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "distributed-tensorflow-guide_amd")

if not isinstance(sys.modules.get("dtg"), type(sys)) or not hasattr(sys.modules.get("dtg"), "__path__"):
    _spec = importlib.util.spec_from_file_location(
        "dtg", os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
    _mod = importlib.util.module_from_spec(_spec)
    sys.modules["dtg"] = _mod
    _spec.loader.exec_module(_mod)
