"""Loader for the native extension ``erasurehead_amd._C``.

The extension (gfx950 HIP kernels + the C++ arrival collector) is built in-tree by
``tools/build_ext.py``; if it is missing it is built on first use (hipcc cross-compiles
without a GPU).  GPU code paths call :func:`native` and fail loudly when the extension
cannot be loaded — there is no silent eager fallback on a GPU.

Build provenance: the library carries the SHA-256 of the ``csrc/`` tree it was compiled
from (``EH_SOURCE_HASH:<hex>``, see ``tools/build_ext.py``).  Before importing it,
:func:`native` reads that hash straight from the ``.so`` file and compares it with the
sources next to it.  A mismatch rebuilds (``build_if_missing=True``) or raises
:class:`StaleBuildError`; a library that was shipped from elsewhere can therefore never
run kernels other than the ones in this tree.  ``ERASUREHEAD_CSRC_DIR`` points the
check at another source tree (tests).
"""
from __future__ import annotations

import importlib
import os
import sys
import threading

_lock = threading.Lock()
_mod = None
_err = None


class StaleBuildError(RuntimeError):
    """The built ``_C`` library does not match the ``csrc/`` sources of this tree."""


def _root() -> str:
    return os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build_ext():
    tools = os.path.join(_root(), "tools")
    if tools not in sys.path:
        sys.path.insert(0, tools)
    import build_ext  # type: ignore

    return build_ext


def build(force: bool = False, verbose: bool = False) -> str:
    return _build_ext().build(force=force, verbose=verbose)


def csrc_dir() -> str:
    return os.environ.get("ERASUREHEAD_CSRC_DIR") or os.path.join(_root(), "csrc")


def provenance() -> dict:
    """{'so': path, 'built_from': hash in the .so (None if missing), 'tree': hash of csrc/, 'fresh': bool}."""
    be = _build_ext()
    so = be.target_path()
    built = be.embedded_hash(so) if os.path.exists(so) else None
    tree = be.source_hash(csrc_dir())
    return {"so": so, "built_from": built, "tree": tree, "fresh": built is not None and built == tree}


def check_fresh() -> dict:
    """Raise :class:`StaleBuildError` unless the built library matches the source tree."""
    p = provenance()
    if not os.path.exists(p["so"]):
        raise StaleBuildError(f"native extension not built ({p['so']} missing): run python tools/build_ext.py")
    if not p["fresh"]:
        raise StaleBuildError(
            f"stale native build: {os.path.basename(p['so'])} was compiled from csrc/ hash "
            f"{(p['built_from'] or 'unknown')[:16]}, the tree is {p['tree'][:16]}; run python tools/build_ext.py")
    return p


def native(build_if_missing: bool = True):
    """Return the loaded ``_C`` module (building it if missing or stale); raise if impossible."""
    global _mod, _err
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            check_fresh()
        except StaleBuildError as e:
            if not build_if_missing or os.environ.get("ERASUREHEAD_NO_BUILD"):
                raise
            _err = e
            build()
            importlib.invalidate_caches()
            check_fresh()
        # torch first: _C links torch's libraries (and its RCCL); initialised in the other order, the
        # process aborts at exit with a corrupted heap ("corrupted size vs. prev_size")
        import torch  # noqa: F401

        try:
            mod = importlib.import_module("erasurehead_amd._C")
        except ImportError as e:
            raise RuntimeError(f"erasurehead_amd native extension not loadable: {e}") from e
        tree = provenance()["tree"]
        if getattr(mod, "SOURCE_HASH", None) != tree:
            raise StaleBuildError(f"loaded _C reports SOURCE_HASH {getattr(mod, 'SOURCE_HASH', None)!r}, "
                                  f"tree is {tree}")
        _mod = mod
        return _mod


def available() -> bool:
    try:
        native()
        return True
    except Exception:
        return False
