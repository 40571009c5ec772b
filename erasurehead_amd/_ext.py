"""Loader for the native extension ``erasurehead_amd._C``.

The extension (gfx950 HIP kernels + the C++ arrival collector) is built in-tree by
``tools/build_ext.py``; if it is missing it is built on first use (hipcc cross-compiles
without a GPU).  GPU code paths call :func:`native` and fail loudly when the extension
cannot be loaded — there is no silent eager fallback on a GPU.
"""
from __future__ import annotations

import importlib
import os
import sys
import threading

_lock = threading.Lock()
_mod = None
_err = None


def _root() -> str:
    return os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(force: bool = False, verbose: bool = False) -> str:
    tools = os.path.join(_root(), "tools")
    if tools not in sys.path:
        sys.path.insert(0, tools)
    import build_ext  # type: ignore

    return build_ext.build(force=force, verbose=verbose)


def native(build_if_missing: bool = True):
    """Return the loaded ``_C`` module (building it if needed); raise if impossible."""
    global _mod, _err
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            _mod = importlib.import_module("erasurehead_amd._C")
            return _mod
        except ImportError as e:  # not built yet
            _err = e
        if not build_if_missing or os.environ.get("ERASUREHEAD_NO_BUILD"):
            raise RuntimeError(f"erasurehead_amd native extension not available: {_err}")
        build()
        importlib.invalidate_caches()
        _mod = importlib.import_module("erasurehead_amd._C")
        return _mod


def available() -> bool:
    try:
        native()
        return True
    except Exception:
        return False
