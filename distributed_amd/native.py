"""Loader for the in-tree native extensions (``_C`` HIP runtime, ``_h5`` checkpoint I/O).

Policy: on a machine with a GPU the HIP path is mandatory — if ``_C`` cannot be
imported (and cannot be built in-tree) we raise instead of silently falling back to
eager PyTorch.  On CPU-only hosts the native module is optional (the torch reference
path runs, e.g. for the gloo multi-process tests).
"""
from __future__ import annotations

import importlib
import threading

import torch

_lock = threading.Lock()
_C = None
_H5 = None
_err = None


def _try_import(name):
    return importlib.import_module(f"distributed_amd.{name}")


class StaleExtensionError(ImportError):
    """The in-tree ``_C`` was built from other sources than the tree's ``csrc/``."""


def check_fresh(so=None, csrc=None) -> None:
    """Raise :class:`StaleExtensionError` if the built ``_C`` (``so``) does not carry the hash
    of the sources in ``csrc`` (default: this tree).  No-op when the sources are absent (an
    installed package) or ``DAMD_ALLOW_STALE=1``."""
    import os
    from pathlib import Path

    from . import _build

    if os.environ.get("DAMD_ALLOW_STALE", "0") == "1":
        return
    csrc = Path(csrc or os.environ.get("DAMD_CSRC_ROOT") or _build.CSRC)
    so = Path(so or (_build.PKG / f"_C{_build.EXT}"))
    if not (csrc / "bindings.cpp").exists() or not so.exists():
        return
    have, want = _build.embedded_hash(so), _build.source_hash(csrc)
    if have != want:
        raise StaleExtensionError(
            f"{so.name} was built from other sources than {csrc} (embedded hash {have and have[:12]}, "
            f"sources {want[:12]}): rebuild with `python -m distributed_amd._build` "
            "(DAMD_ALLOW_STALE=1 runs it anyway)")


def load_C(build_if_missing: bool = True):
    global _C, _err
    with _lock:
        if _C is not None:
            return _C
        try:
            check_fresh()  # before the import: a loaded extension cannot be replaced
        except StaleExtensionError:
            if not build_if_missing:
                raise
            from . import _build

            _build._build_C()
            check_fresh()
        try:
            _C = _try_import("_C")
        except ImportError as e:  # not built yet
            _err = e
            if build_if_missing:
                from . import _build

                _build._build_C()
                _C = _try_import("_C")
        return _C


def load_h5(build_if_missing: bool = True):
    global _H5
    with _lock:
        if _H5 is not None:
            return _H5
        try:
            _H5 = _try_import("_h5")
        except ImportError:
            if not build_if_missing:
                raise
            from . import _build

            _build._build_h5()
            _H5 = _try_import("_h5")
        return _H5


def gpu_available() -> bool:
    return torch.cuda.is_available()


def require_C():
    """Native module or a loud failure (used by every GPU code path)."""
    try:
        return load_C()
    except Exception as e:  # pragma: no cover - exercised on broken installs only
        raise RuntimeError(
            "distributed_amd native extension (_C) is unavailable; the GPU path has no "
            f"eager fallback. Build it with `python -m distributed_amd._build`: {e}"
        ) from e


def native_status() -> dict:
    st = {"gpu": gpu_available(), "C": False, "h5": False}
    try:
        load_C(build_if_missing=False)
        st["C"] = True
    except Exception as e:
        st["C_error"] = repr(e)
    try:
        load_h5(build_if_missing=False)
        st["h5"] = True
    except Exception as e:
        st["h5_error"] = repr(e)
    return st
