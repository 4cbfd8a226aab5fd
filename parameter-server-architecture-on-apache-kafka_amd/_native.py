"""Loader for the in-tree native extensions.

``_psx_host`` (C++ host runtime) is always required.  ``_psx_hip`` (HIP
kernels) is required whenever a GPU is used: :func:`hip` raises instead of
silently falling back to PyTorch, so a GPU run can never pass on an eager
fallback path.
"""
from __future__ import annotations

import importlib
import os

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
_hip_mod = None
_hip_err = None


def _build_hint() -> str:
    return "build the native extensions first: python csrc/build.py (or python -c 'import __graft_entry__ as g; g.build()')"


try:
    from . import _psx_host as host  # type: ignore
except ImportError as e:  # pragma: no cover - build problem
    raise ImportError(f"psx native host runtime missing ({e}); {_build_hint()}") from e


def hip():
    """Return the HIP extension module, importing torch first so the HIP runtime
    symbols bind to the libamdhip64 that torch already loaded."""
    global _hip_mod, _hip_err
    if _hip_mod is not None:
        return _hip_mod
    import torch  # noqa: F401

    try:
        _hip_mod = importlib.import_module(__package__ + "._psx_hip")
    except ImportError as e:
        _hip_err = e
        raise RuntimeError(f"psx HIP extension (_psx_hip) failed to load: {e}; {_build_hint()}") from e
    return _hip_mod


def hip_loaded_path() -> str | None:
    return getattr(_hip_mod, "__file__", None)
