"""Loader for the C++ runtime module ``_dryad_native`` (built in-tree by ``dryad_amd._build``)."""
from __future__ import annotations

import importlib.util
import os
import threading

from ._build import build_runtime, runtime_lib_path

_MOD = None
_LOCK = threading.Lock()


def runtime():
    """Return the loaded pybind11 runtime module (builds it on first use when missing)."""
    global _MOD
    if _MOD is not None:
        return _MOD
    with _LOCK:
        if _MOD is not None:
            return _MOD
        path = runtime_lib_path()
        if not path.exists() and os.environ.get("DRYAD_AUTOBUILD", "1") == "1":
            build_runtime()
        if not path.exists():
            raise ImportError(f"{path} missing: run `python -m dryad_amd._build`")
        spec = importlib.util.spec_from_file_location("_dryad_native", str(path))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _MOD = mod
        return mod
